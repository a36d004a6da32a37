"""Correction factors from tools/probe/fetch_calib runs: known bytes / counter bytes per shape.
    python tools/probe/fetch_calib.py FETCH_DIR WRITE_DIR"""
import csv
import glob
import sys

BYTES = 1 << 30
SEG = (BYTES // 576 // 16) * 16 * 576
SHAPES = [("rd<HIP_vector_type<unsigned int, 4u", "rd16", BYTES),
          ("rd<HIP_vector_type<unsigned int, 2u", "rd8", BYTES), ("rd<unsigned int>", "rd4", BYTES),
          ("seg64", "seg64", SEG), ("dma16", "dma16", BYTES),
          ("wr<HIP_vector_type<unsigned int, 4u", "wr16", BYTES),
          ("wr<HIP_vector_type<unsigned int, 2u", "wr8", BYTES), ("wseg64", "wseg64", SEG)]


def load(d, counter):
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"]) * 1024))
    return sorted(rows)


def main():
    for d, counter in ((sys.argv[1], "FETCH_SIZE"), (sys.argv[2], "WRITE_SIZE")):
        rows = load(d, counter)
        print(f"{counter}:")
        # dispatch 1 is hipMemset's fill; then a flush sweep (wr<uint4> over the other buffer)
        # before each measured kernel
        measured = [r for r in rows if "fillBuffer" not in r[1]][1::2]
        for (_, name, val), (pat, label, known) in zip(measured, SHAPES):
            assert pat in name, (pat, name)
            print(f"  {label:8s} counter {val / 2**20:10.1f} MiB  known {known / 2**20:8.1f} MiB  "
                  f"known/counter = {known / max(val, 1):.3f}")


if __name__ == "__main__":
    main()
