"""Static audit of MFMA result hazards in libhvk's gfx950 ISA (hipcc --save-temps output).

hipcc (ROCm 7.2) pads the "XDL MFMA writes a VGPR -> a later instruction reads or writes it"
hazard within a basic block, but a reader at a BRANCH TARGET whose predecessor ends right
after the MFMA was found padded with 2 states instead of 8 (wmsa_ring.hip: the unmasked-window
path skipping the mask block read the scores too early; wrong values, no fault).  This walks
every path from each MFMA (fallthrough and taken branches) and reports any instruction that
touches the MFMA's destination registers within MIN_STATES wait states (an MFMA taking the
whole destination as its accumulator C is the legal chain and is skipped, and so is the same
MFMA opcode overwriting without reading part of the destination: XDL results retire in issue
order; the remaining registers stay watched).

    python tools/mfma_hazard_audit.py [--states 8] file.hip ...   (default: every csrc/*.hip)
"""
import argparse
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "hierarchical-vision_amd", "csrc")
REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def parse(asm):
    """-> {kernel: (lines, labels)} with lines = [(mnemonic, operand text)]."""
    kernels, cur = {}, None
    for raw in asm.splitlines():
        line = raw.split(";")[0].rstrip()
        if not line.strip():
            continue
        if re.match(r"^[A-Za-z_.$][\w.$]*:", line) and not line.startswith("\t"):
            name = line.split(":")[0]
            if not name.startswith("."):
                cur = name
                kernels[cur] = ([], {})
                continue
            if cur is not None:
                kernels[cur][1][name] = len(kernels[cur][0])
            continue
        if cur is None or line.strip().startswith("."):
            continue
        parts = line.strip().split(None, 1)
        kernels[cur][0].append((parts[0], parts[1] if len(parts) > 1 else ""))
        if parts[0] == "s_endpgm":
            cur = None
    return kernels


def states(mn, ops):
    if mn == "s_nop":
        return int(ops.strip(), 0) + 1
    return 1


SREG = re.compile(r"^s\[(\d+):(\d+)\]$|^s(\d+)$")


def sregs(op):
    m = SREG.match(op)
    if not m:
        return set()
    if m.group(3) is not None:
        return {int(m.group(3))}
    return set(range(int(m.group(1)), int(m.group(2)) + 1))


def branch_facts(mn, f, known, vcc):
    """Path facts for the structurizer's flag idiom (`s_mov_b64 sX, 0 / -1` on one arm, then
    `s_andn2_b64 vcc, exec, sX` + `s_cbranch_vccnz`): -> (known, vcc, only) where known maps an
    SGPR pair to the constant this path last wrote to it, vcc is "nz" / "z" / None (unknown), and
    only is "taken" / "fall" when this is a branch whose direction the path fixes.  exec is taken
    as non-zero: with exec = 0 no vector write happens, so no hazard is lost."""
    dst = f[0] if f else ""
    if mn.startswith("s_") and not mn.startswith(("s_cbranch", "s_branch", "s_waitcnt", "s_nop")):
        w = sregs(dst)  # any scalar write forgets the pairs it overlaps
        known = {k: v for k, v in known.items() if not (sregs(k) & w)}
    if mn == "s_mov_b64" and SREG.match(dst) and f[1:2] in (["0"], ["-1"]):
        return {**known, dst: int(f[1])}, vcc, None
    if mn in ("s_andn2_b64", "s_and_b64") and f[:2] == ["vcc", "exec"] and len(f) == 3 and f[2] in known:
        zero = known[f[2]] == (0 if mn == "s_and_b64" else -1)
        return known, ("z" if zero else "nz"), None
    if mn in ("s_cbranch_vccnz", "s_cbranch_vccz"):
        if vcc is None:
            return known, vcc, None
        return known, vcc, "taken" if (vcc == "nz") == (mn == "s_cbranch_vccnz") else "fall"
    if "vcc" in f or mn.startswith("v_cmp"):  # anything else that may write vcc
        vcc = None
    return known, vcc, None


def audit(lines, labels, min_states):
    bad = []
    for i, (mn, ops) in enumerate(lines):
        if not mn.startswith("v_mfma"):
            continue
        fields = [f.strip() for f in ops.split(",")]
        seen = set()
        work = [(i + 1, 0, frozenset(regs(fields[0])), {}, None)]
        while work:
            j, st, dst, known, vcc = work.pop()
            while j < len(lines) and st < min_states and dst:
                key = (j, st, dst, frozenset(known.items()), vcc)
                if key in seen:
                    break
                seen.add(key)
                m2, o2 = lines[j]
                f2 = [f.strip() for f in o2.split(",")]
                known, vcc, only = branch_facts(m2, f2, known, vcc)
                touched = regs(o2) & dst
                if touched:
                    is_mfma = m2.startswith("v_mfma") and len(f2) >= 4
                    reads = (regs(f2[1]) | regs(f2[2]) | regs(f2[3])) & dst if is_mfma else touched
                    if is_mfma and regs(f2[3]) == dst and not ((regs(f2[1]) | regs(f2[2])) & dst):
                        break  # the accumulation chain: C = the whole earlier destination
                    if is_mfma and not reads and m2 == mn:
                        # the same XDL opcode overwriting (not reading) part of the destination:
                        # XDL results retire in issue order, so the later write wins (LLVM's
                        # hazard recognizer pads no XDL -> XDL write-after-write of equal passes);
                        # the earlier MFMA's remaining registers stay under watch
                        dst = dst - frozenset(regs(f2[0]))
                    else:
                        bad.append((i, j, st, mn, m2 + " " + o2))
                        break
                if m2 == "s_endpgm":
                    break
                if m2.startswith("s_cbranch") or m2 == "s_branch":
                    tgt = labels.get(o2.strip())
                    if tgt is not None and only != "fall":
                        work.append((tgt, st + 1, dst, known, vcc))
                    if m2 == "s_branch" or only == "taken":
                        break
                st += states(m2, o2)
                j += 1
    return bad


def asm_of(path):
    with tempfile.TemporaryDirectory() as d:
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
                        "-I", CSRC, "-c", os.path.abspath(path), "-o", os.path.join(d, "x.o"), "--save-temps"],
                       cwd=d, check=True, capture_output=True)
        s = [f for f in os.listdir(d) if f.endswith("gfx950.s")]
        with open(os.path.join(d, s[0])) as f:
            return f.read()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--states", type=int, default=8)
    ap.add_argument("files", nargs="*")
    a = ap.parse_args()
    files = a.files or sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    return report(files, a.states)


def report(files, min_states=8, jobs=8):
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(jobs) as ex:
        asms = list(ex.map(asm_of, files))
    total = 0
    for f, asm in zip(files, asms):
        for k, (lines, labels) in parse(asm).items():
            for i, j, st, mn, what in audit(lines, labels, min_states):
                total += 1
                print(f"{os.path.basename(f)}: {k[:70]}: {mn} @{i} -> @{j} after {st} states: {what}")
    print(f"{total} hazard(s) below {min_states} states")
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
