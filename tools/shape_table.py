"""The per-shape GEMM binding-roof table of a bench.py JSON line (mfma.shapes / mfma.binding) as
text, sorted by time per step:  python tools/shape_table.py bench.json > gemm_shapes.txt"""
import json
import sys


def main():
    d = json.load(open(sys.argv[1]))
    m = d["mfma"]
    print("per-shape GEMM binding-roof table (bench.py mfma.shapes, in-step, dispatch-packet timed)")
    print(f"binding: {m['binding']}")
    print(f"{'kernel':18s} {'M':>7s} {'N':>5s} {'K':>5s} wgrad n/step  avg_us roof_us bound   frac ms/step")
    for s in sorted(m["shapes"], key=lambda s: -s["ms_per_step"]):
        print(f"{s['kernel']:18s} {s['M']:7d} {s['N']:5d} {s['K']:5d} {int(s['wgrad']):5d} {s['launches_per_step']:6.2f} "
              f"{s['avg_us']:7.1f} {s['roof_us']:7.1f} {s['bound']:5s} {s['binding_frac']:6.3f} {s['ms_per_step']:7.3f}")


if __name__ == "__main__":
    main()
