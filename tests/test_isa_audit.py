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
