"""bench.py's accounting helpers on the CPU: the W-MSA algorithmic work per step (SURVEY.md
§8(d)), the kernel labels, and the roofline block's choice of roof (HBM below the 312 flop/B
ridge, MFMA above it)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_wmsa_work_swinv2_tiny():
    import bench
    from hvamd import swinv2
    net = swinv2.SwinTransformerV2(img_size=224, embed_dim=96, depths=[2, 2, 6, 2],
                                   num_heads=[3, 6, 12, 24], window_size=7, num_classes=10)
    w = bench.wmsa_work(net, 256)
    # sum over blocks of T*C per image = 1 430 016: 8 B / 16 B per element
    assert w["fwd_bytes"] == 8 * 1430016 * 256 == 2928672768
    assert w["bwd_bytes"] == 2 * w["fwd_bytes"]
    assert w["fwd_flops"] == 4 * 49 * 1430016 * 256  # 4 T N C, N = 49 tokens per window
    assert w["windows"] == {7}


def test_kernel_names():
    import bench
    assert bench.kernel_names({7}) == ("wmsa_fwd_win_kernel<7,HG>+ring", "wmsa_bwd_pair_kernel<7>")
    f, b = bench.kernel_names({12, 24})
    assert f == "wmsa_fwd_large_kernel<12>+wmsa_fwd_large_kernel<24>"
    assert b == "wmsa_bwd_large_kernel<12>+wmsa_bwd_large_kernel<24>"


@pytest.mark.parametrize("ai,bound", [(24.5, "hbm"), (351.0, "mfma")])
def test_roofline_block_picks_the_binding_roof(ai, bound):
    import bench
    nbytes = 1_000_000_000
    flops = int(ai * nbytes)
    r = bench.roofline_block("k", nbytes, flops, ms_total=2.0, launches=4, steps=2, traffic=None)
    assert r["bound"] == bound
    gbs = nbytes * 2 / 2e-3 / 1e9
    tfs = flops * 2 / 2e-3 / 1e12
    assert r["achieved_gbs"] == pytest.approx(gbs, rel=1e-6)
    assert r["hbm_frac"] == pytest.approx(gbs / bench.HBM_PEAK_GBS, abs=1e-4)
    assert r["mfma_frac"] == pytest.approx(tfs / bench.MFMA_PEAK_TFS, abs=1e-4)
    if bound == "hbm":
        assert r["unit"] == "GB/s" and r["frac"] == r["hbm_frac"]
    else:
        assert r["unit"] == "TFLOP/s" and r["frac"] == r["mfma_frac"]
    assert r["avg_launch_us"] == pytest.approx(500.0)
    assert r["ms_per_step"] == pytest.approx(1.0)
