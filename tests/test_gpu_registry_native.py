"""Every registered SwinV2 (hvamd.models.MODEL_REGISTRY, the reference's timm names,
/root/reference/models.py:16-51) runs its forward and backward on libhvk only: one bf16-autocast
train pass at batch 1 under options.strict_native (a launch that would leave libhvk raises) and
zero counted library fallbacks.  Guards the per-model shape tables (e.g. SwinV2-B's 128-wide patch
embedding, whose weight gradient had no kernel variant before round 6)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["swinv2_tiny_window7_224", "swinv2_small_window7_224",
                                  "swinv2_base_window7_224", "swinv2_tiny_window8_256",
                                  "swinv2_base_window8_256", "swinv2_base_window24_384"])
def test_registry_model_runs_native_only(name):
    from hvamd import models, ops, options
    torch.manual_seed(0)
    net = models.create_model(name, num_classes=1000, drop_path_rate=0.0).cuda().train()
    x = torch.randn(1, 3, net.patch_embed.img_size[0], net.patch_embed.img_size[1], device="cuda")
    ops.library_fallbacks(reset=True)
    with options.override(strict_native=True):
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = net(x)
        y.float().square().mean().backward()
    torch.cuda.synchronize()
    assert ops.library_fallbacks(reset=True) == {}
    assert torch.isfinite(y.float()).all()
    bad = [k for k, p in net.named_parameters() if p.requires_grad and (p.grad is None or not torch.isfinite(p.grad).all())]
    assert not bad, bad[:5]
