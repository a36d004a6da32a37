"""MFMA busy fraction and effective clock per kernel category from one rocprofv3 PMC pass
(SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CU_CYCLES, GRBM_GUI_ACTIVE) over a short bench run:

    python tools/mfma_pmc.py DIR OUT.json

effective clock = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs) / kernel duration
(MI355X_MICROARCH.md, DVFS give-back); MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (cycles x 1024
SIMDs), with cycles = GRBM_GUI_ACTIVE / 8: the fraction of SIMD-cycles the matrix cores were
busy while the kernel ran (a 2.5 PF peak assumes 2.4 GHz; at the measured clock the dense
peak is clock / 2.4 GHz x 2.5 PF)."""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.kernel_summary import category  # noqa: E402


def main():
    d, out = sys.argv[1], sys.argv[2]
    rows = collections.defaultdict(dict)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Kernel_Name"])
            rows[key][r["Counter_Name"]] = rows[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    dur = {}
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    agg = collections.defaultdict(lambda: [0.0, 0.0, 0.0, 0])
    for (did, name), c in rows.items():
        if did not in dur or "GRBM_GUI_ACTIVE" not in c:
            continue
        a = agg[category(name)]
        a[0] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        a[1] += c["GRBM_GUI_ACTIVE"] / 8
        a[2] += dur[did]
        a[3] += 1
    res = {}
    for k, (busy, cyc, t, n) in sorted(agg.items(), key=lambda kv: -kv[1][2]):
        res[k] = {"launches": n, "seconds": round(t, 6), "effective_clock_ghz": round(cyc / t / 1e9, 3) if t else None,
                  "mfma_busy_frac": round(busy / (cyc * 1024), 4) if cyc else None}
        print(f"{k:12s} {n:5d} launches {t * 1e3:8.3f} ms  clock {res[k]['effective_clock_ghz']} GHz  "
              f"MFMA busy {res[k]['mfma_busy_frac']}")
    json.dump({"source": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE "
                         "--kernel-trace over bench.py --steps 2 --warmup 1", "categories": res},
              open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
