"""Device-side input normalisation (data.py:130-136, composer NormalizationFn) on libhvk:
bit-exact against torch's own f32 sub_ / div_ (then the bf16 cast the autocast conv applies)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

MEAN = [0.463 * 255, 0.480 * 255, 0.376 * 255]  # configs.py:30-31 scaled as data.py:128-133
STD = [0.238 * 255, 0.229 * 255, 0.247 * 255]


def _u8(B, H, W, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.randint(0, 256, (B, 3, H, W), generator=g, device="cuda", dtype=torch.uint8)


def _torch_norm(x):
    m = torch.tensor(MEAN, device="cuda").view(1, 3, 1, 1)
    s = torch.tensor(STD, device="cuda").view(1, 3, 1, 1)
    return x.float().sub_(m).div_(s)


@pytest.mark.parametrize("B,H,W", [(2, 224, 224), (3, 32, 48), (1, 384, 384)])
def test_normalize_u8_bit_exact(B, H, W):
    from hvamd.data import NormalizationFn
    x = _u8(B, H, W)
    y, _ = NormalizationFn(MEAN, STD)((x, None))
    assert y.dtype == torch.float32 and torch.equal(y, _torch_norm(x))


@pytest.mark.parametrize("B,H,W", [(2, 224, 224), (3, 32, 48)])
def test_patchify_u8_fused_bit_exact(B, H, W):
    import hvamd.ops as ops
    x = _u8(B, H, W, 1)
    mean, std = torch.tensor(MEAN, device="cuda"), torch.tensor(STD, device="cuda")
    out = ops.patchify_u8_bf16(x, 4, mean, std)
    ref = _torch_norm(x).bfloat16().reshape(B, 3, H // 4, 4, W // 4, 4).permute(0, 2, 4, 1, 3, 5)
    assert torch.equal(out, ref.reshape(B, -1, 48))


def test_fused_normalization_model_equals_transform_then_model():
    """A NormalizationFn handed to the Trainer is folded into PatchEmbed (uint8 batch straight
    to the model): logits bit-identical to normalising first (the reference's device
    transform) and feeding the f32 images."""
    from hvamd import hierarchy, models, optim, swinv2
    from hvamd.data import NormalizationFn
    from hvamd.trainer import Trainer
    torch.manual_seed(0)
    net = swinv2.SwinTransformerV2(img_size=56, embed_dim=32, depths=[2, 2], num_heads=[1, 2],
                                   window_size=7, num_classes=10, drop_path_rate=0.0).cuda().eval()
    x = _u8(2, 56, 56, 2)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        ref = net(_torch_norm(x))
    model = models.Model(net, None, None, hierarchy.soft_cross_entropy)
    opt = optim.DecoupledSGDW(optim.set_weight_decay(model), lr=0.0, momentum=0.9)
    t = Trainer(model, opt, device_transforms=NormalizationFn(MEAN, STD))
    assert t.device_transforms is None and net.patch_embed.input_norm is not None
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        mine = net(x)
    assert torch.equal(mine, ref)
    loss = t.train_step((x, torch.tensor([1, 2], device="cuda")))
    assert torch.isfinite(loss)
