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
    assert bench.kernel_names({7}) == ("wmsa_fwd_win_kernel<7,HG>", "wmsa_bwd_pair_kernel<7>")
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


def test_stage_breakdown_groups_launches_by_block_resolution():
    """bench.py's per-stage view: launch i of a step belongs to block i mod 12 (forward order;
    the backward in reverse), grouped by resolution with the per-launch bytes of SURVEY.md §8(d)."""
    import bench
    from hvamd import swinv2
    net = swinv2.SwinTransformerV2(img_size=224, embed_dim=96, depths=[2, 2, 6, 2],
                                   num_heads=[3, 6, 12, 24], window_size=7, num_classes=10)
    per_stage_us = [100.0, 50.0, 30.0, 20.0]
    fwd = [per_stage_us[s] / 1000 for s in [0, 0, 1, 1, 2, 2, 2, 2, 2, 2, 3, 3]] * 3  # 3 steps
    st = bench.stage_breakdown(net, 256, fwd, 8, backward=False)
    assert [g["resolution"] for g in st] == [[56, 56], [28, 28], [14, 14], [7, 7]]
    assert [g["launches_per_step"] for g in st] == [2, 2, 6, 2]
    assert [g["avg_launch_us"] for g in st] == per_stage_us
    assert st[0]["bytes_per_launch"] == 8 * 256 * 56 * 56 * 96
    assert st[0]["achieved_gbs"] == pytest.approx(8 * 256 * 56 * 56 * 96 / 100e-6 / 1e9, rel=1e-3)
    bwd = fwd[::-1]  # the backward launches stage 3 first
    sb = bench.stage_breakdown(net, 256, bwd, 16, backward=True)
    assert [g["avg_launch_us"] for g in sb] == per_stage_us
    assert bench.stage_breakdown(net, 256, fwd[:5], 8, backward=False) is None
