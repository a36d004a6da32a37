"""Static checks of libhvk's gfx950 machine code (CPU only: hipcc cross-compiles)."""
import glob
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="needs hipcc")
def test_no_mfma_result_hazard_on_any_path():
    """Every path from every MFMA (fallthrough and taken branches) leaves >= 8 wait states before
    an instruction touches its destination (hipcc misses the taken-branch case, hvk_common.h
    hvk_settle); an MFMA accumulating into the whole destination is the legal chain."""
    import mfma_hazard_audit as audit
    files = sorted(glob.glob(os.path.join(ROOT, "hierarchical-vision_amd", "csrc", "*.hip")))
    assert audit.report(files, 8, jobs=min(8, os.cpu_count() or 1)) == 0


def _audit_asm(body):
    import mfma_hazard_audit as audit
    asm = "k:\n" + "\n".join("\t" + l if not l.startswith(".") else l for l in body) + "\n\ts_endpgm\n"
    lines, labels = audit.parse(asm)["k"]
    return audit.audit(lines, labels, 8)


def test_audit_flags_taken_branch_reader():
    """Positive control: a reader at a branch target 2 states after the MFMA is reported."""
    bad = _audit_asm(["v_mfma_f32_16x16x32_bf16 v[0:3], v[4:7], v[8:11], v[0:3]",
                      "s_cbranch_scc1 .LBB0_1", "s_nop 7", ".LBB0_1:", "v_add_f32_e32 v12, v0, v1"])
    assert len(bad) == 1 and "v_add_f32" in bad[0][4]


def test_audit_follows_structurizer_flags():
    """The arm that sets the flag pair to 0 always takes `s_andn2_b64 vcc, exec, flag` +
    `s_cbranch_vccnz` past the other arm's reader (wmsa_large.hip w12, ROCm 7.2); with the flag
    at -1 on the path the fallthrough reader is still reported."""
    def body(flag):
        return ["v_mfma_f32_16x16x32_bf16 v[0:3], v[4:7], v[8:11], v[12:15]",
                f"s_mov_b64 s[20:21], {flag}", "s_andn2_b64 vcc, exec, s[20:21]",
                "s_cbranch_vccnz .LBB0_2", "ds_read_b128 v[0:3], v16", ".LBB0_2:", "s_nop 7"]
    assert _audit_asm(body(0)) == []
    assert len(_audit_asm(body(-1))) == 1
