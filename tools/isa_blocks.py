"""Per-basic-block instruction mix of one kernel in a hipcc --save-temps .s file.

    python tools/isa_blocks.py FILE.s KERNEL_REGEX [--min N]

Prints each block's instruction count by class (VALU, transcendental, MFMA, SALU, LDS, VMEM,
waitcnt / nop) and where it branches, plus the kernel's register / LDS budget -- the numbers
used to read a loop body's issue cost."""
import argparse
import re

TRANS = ("v_exp_", "v_log_", "v_rcp_", "v_rsq_", "v_sqrt_", "v_sin_", "v_cos_")


def classify(op):
    if "mfma" in op:
        return "mfma"
    if op.startswith(TRANS):
        return "trans"
    if op.startswith("v_accvgpr"):
        return "acc"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_sleep")):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("file")
    ap.add_argument("kernel")
    ap.add_argument("--min", type=int, default=20, help="only blocks with at least this many instructions")
    a = ap.parse_args()
    lines = open(a.file).read().split("\n")
    pat = re.compile(a.kernel)
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S+:", l) and pat.search(l.split(":")[0]))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    name = lines[start].split(":")[0]
    print(name)
    body = lines[start:end]
    cur, rows, tot = "entry", [], {}
    counts, last = {}, ""
    for l in body[1:] + [".LBBend:"]:
        m = re.match(r"^(\.LBB\d+_\d+|\.LBBend):", l)
        if m:
            rows.append((cur, counts, last))
            cur, counts, last = m.group(1), {}, ""
            continue
        t = l.strip()
        if not t or t.startswith((".", ";")):
            continue
        op = t.split()[0]
        c = classify(op)
        counts[c] = counts.get(c, 0) + 1
        tot[c] = tot.get(c, 0) + 1
        if op.startswith("s_cbranch") or op.startswith("s_branch"):
            last = t
    for blk, c, br in rows:
        n = sum(c.values())
        if n >= a.min:
            print(f"{blk:14s} {n:5d}  " + " ".join(f"{k}={v}" for k, v in sorted(c.items())) + (f"   -> {br}" if br else ""))
    print("total", sum(tot.values()), " ".join(f"{k}={v}" for k, v in sorted(tot.items())))
    meta = "\n".join(lines[end:end + 400])
    for key in ("vgpr_count", "agpr_count", "sgpr_count", "group_segment_fixed_size", "private_segment_fixed_size"):
        m = re.search(rf"\.{key}:\s+(\d+)", meta)
        if m:
            print(f"  {key} {m.group(1)}")


if __name__ == "__main__":
    main()
