"""Per-kernel averages of rocprofv3 --pmc counter CSVs:  python tools/pmc_report.py DIR [regex]"""
import collections
import csv
import glob
import re
import sys


def main():
    d = sys.argv[1]
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if pat and not pat.search(k):
                continue
            agg[k[:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(k)
        for c in sorted(v):
            vals = v[c]
            print(f"    {c:28s} {sum(vals) / len(vals):16.0f}   (n={len(vals)})")


if __name__ == "__main__":
    main()
