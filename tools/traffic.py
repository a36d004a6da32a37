"""HBM traffic per launch of the W-MSA kernels from two rocprofv3 PMC passes over a short
bench.py run (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950):
    python tools/traffic.py FETCH_DIR WRITE_DIR [OUT.json]
Corrections (MI355X_MICROARCH.md, HBM; calibrated on this box class by tools/probe/fetch_calib,
profiles/round3/fetch_calib.txt): FETCH_SIZE counts half the bytes of coalesced streaming reads
of 4, 8 and 16 B per lane and of LDS-DMA -> x2; two thirds of them for an isolated 64-B-segment
shape (x1.5, seg64: segments of one 128-B line fetched as separate requests).  The W-MSA reads
use x2: at x1.5 the backward's count falls below its algorithmic bytes (impossible for a
first read), i.e. its segments merge into whole-line requests.  WRITE_SIZE is exact for
4-16-B stores.  Both counters are in KiB."""
import collections
import csv
import glob
import json
import sys

# the forward: wmsa_fwd_win_kernel (the ring form when selected for A/B runs)
KERNELS = {"wmsa_fwd": ("wmsa_fwd_win_kernel", "wmsa_fwd_ring_kernel"), "wmsa_bwd": ("wmsa_bwd_pair_kernel",),
           "mlp_fwd": ("mlp_fwd_kernel",), "mlp_bwd": ("mlp_bwd_kernel",)}  # the last two: fused stage-0 MLP


def per_kernel(d, counter):
    out = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            for key, pats in KERNELS.items():
                if any(p in r["Kernel_Name"] for p in pats):
                    out[key].append(float(r["Counter_Value"]))
    return out


def main():
    fetch, write = per_kernel(sys.argv[1], "FETCH_SIZE"), per_kernel(sys.argv[2], "WRITE_SIZE")
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) over "
                     "bench.py --steps 2 --warmup 1; FETCH_SIZE x2 (gfx950 16-B/lane reads), KiB -> B",
           "kernels": {}}
    for key in KERNELS:
        f, w = fetch.get(key, []), write.get(key, [])
        if not f or not w:
            continue
        fb = 2 * 1024 * sum(f) / len(f)
        wb = 1024 * sum(w) / len(w)
        res["kernels"][key] = {"launches": len(f), "fetch_bytes_per_launch": round(fb),
                               "write_bytes_per_launch": round(wb),
                               "traffic_bytes_per_launch": round(fb + wb)}
    s = json.dumps(res, indent=1)
    print(s)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(s + "\n")


if __name__ == "__main__":
    main()
