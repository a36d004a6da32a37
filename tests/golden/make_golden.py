"""Generate the golden fixtures under tests/golden/ by importing the REFERENCE
(/root/reference, read-only) in the build container.

Run:  python tests/golden/make_golden.py [--only index,modules,models,taxonomy,losses,swinb,prod,steps,prodb,step256]
      (needs /root/reference; CPU only)

The reference's third-party imports that are absent offline are replaced by
minimal stand-ins installed into sys.modules before import:
  * timm.models.layers: DropPath (identity; all goldens use drop_path=0),
    to_2tuple, trunc_normal_   (swinv2.py:9)
  * composer.metrics.CrossEntropy, torchmetrics.Metric,
    torchvision.datasets.ImageFolder  (hierarchy.py:6-15; only used as base
    classes -- none of the functions exercised here touch them)
Every array written is data (inputs and the reference's outputs); no reference
source is copied into the repo.
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("HV_REFERENCE", "/root/reference")


def install_shims():
    timm = types.ModuleType("timm")
    tm = types.ModuleType("timm.models")
    tml = types.ModuleType("timm.models.layers")

    class DropPath(torch.nn.Module):
        def __init__(self, p=0.0):
            super().__init__()
            self.p = p

        def forward(self, x):
            assert not self.training or self.p == 0.0
            return x

    tml.DropPath = DropPath
    tml.to_2tuple = lambda x: tuple(x) if isinstance(x, (list, tuple)) else (x, x)
    tml.trunc_normal_ = lambda t, std=1.0, **k: torch.nn.init.trunc_normal_(t, std=std)
    sys.modules.update({"timm": timm, "timm.models": tm, "timm.models.layers": tml})

    composer = types.ModuleType("composer")
    cm = types.ModuleType("composer.metrics")

    class CrossEntropy:  # placeholder base class
        pass

    cm.CrossEntropy = CrossEntropy
    composer.metrics = cm
    sys.modules.update({"composer": composer, "composer.metrics": cm})

    tmx = types.ModuleType("torchmetrics")

    class Metric(torch.nn.Module):
        pass

    tmx.Metric = Metric
    sys.modules["torchmetrics"] = tmx
    tv = types.ModuleType("torchvision")
    tvd = types.ModuleType("torchvision.datasets")

    class ImageFolder:
        pass

    tvd.ImageFolder = ImageFolder
    tv.datasets = tvd
    sys.modules.update({"torchvision": tv, "torchvision.datasets": tvd})


def sampled(name, a, n=8192):
    """Deterministic subset of a large array (index draw from numpy default_rng seeded by
    crc32(name), restated by tests/golden_util.py): a parity check on n entries keeps the
    fixture small where the full tensor is hundreds of KB of incompressible floats."""
    import zlib
    a = np.asarray(a, np.float32).reshape(-1)
    if a.size <= n:
        return a
    idx = np.random.default_rng(zlib.crc32(name.encode())).choice(a.size, n, replace=False)
    return a[np.sort(idx)]


def seeded(seed, shape):
    """Inputs the tests regenerate instead of storing: standard normals, f32."""
    return np.random.default_rng(seed).standard_normal(shape).astype(np.float32)


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="index,modules,models,taxonomy,losses,swinb,prod")
    only = set(ap.parse_args().only.split(","))
    install_shims()
    sys.path.insert(0, REF)
    sys.path.insert(0, REPO)
    import hierarchy as ref_h  # noqa: E402  (reference)
    import swinv2 as ref  # noqa: E402  (reference)
    from oracle.hierarchy_ref import synthetic_inat_names
    from oracle.swinv2_ref import init_params_from_rng

    torch.manual_seed(0)
    torch.set_num_threads(min(8, os.cpu_count() or 1))

    if "swinb" in only:
        swinb_and_prod(ref, init_params_from_rng, "swinb")
    if "prod" in only:
        swinb_and_prod(ref, init_params_from_rng, "prod")
    if "steps" in only:
        train_steps(ref, ref_h, init_params_from_rng)
    if "prodb" in only:
        bench_batch_modules(ref, init_params_from_rng)
    if "step256" in only:
        train_step_b256(ref, init_params_from_rng)
    if "index" not in only:
        return main_rest(ref, ref_h, only)
    # ---------------------------------------------------------------- indices
    idx = {}
    for w, pws in [(7, [0, 12]), (8, [0]), (12, [0, 12]), (24, [0, 12, 6]), (6, [0])]:
        for pw in pws:
            wa = ref.WindowAttention(dim=32, window_size=(w, w), num_heads=1,
                                     pretrained_window_size=(pw, pw))
            idx[f"rpi_w{w}"] = wa.relative_position_index.numpy()
            idx[f"coords_w{w}_pw{pw}"] = wa.relative_coords_table.numpy()
    for res, w, s in [(56, 7, 3), (28, 7, 3), (14, 7, 3), (7, 7, 3), (56, 7, 0),
                      (96, 24, 12), (48, 24, 12), (24, 24, 12), (12, 24, 12),
                      (64, 8, 4), (16, 8, 4)]:
        blk = ref.SwinTransformerBlock(dim=32, input_resolution=(res, res), num_heads=1,
                                       window_size=w, shift_size=s)
        ew, es = blk.window_size, blk.shift_size
        key = f"r{res}_w{w}_s{s}"
        idx[key + "_eff"] = np.array([ew, es], np.int64)
        idx[key + "_mask"] = (blk.attn_mask.numpy() if blk.attn_mask is not None
                              else np.zeros((0,), np.float32))
        img = torch.arange(res * res, dtype=torch.float64).reshape(1, res, res, 1)
        if es > 0:
            img = torch.roll(img, shifts=(-es, -es), dims=(1, 2))
        win = ref.window_partition(img, ew).reshape(-1, ew * ew)
        idx[key + "_gather"] = win.numpy().astype(np.int32)
    for res in [56, 28, 14, 96, 48, 24]:
        pm = ref.PatchMerging((res, res), dim=1)
        pm.reduction = torch.nn.Identity()
        pm.norm = torch.nn.Identity()
        x = torch.arange(res * res, dtype=torch.float64).reshape(1, res * res, 1)
        idx[f"merge_r{res}"] = pm(x)[0].numpy().astype(np.int32)
    np.savez_compressed(os.path.join(HERE, "index_golden.npz"), **idx)
    main_rest(ref, ref_h, only)


def main_rest(ref, ref_h, only):
    from oracle.hierarchy_ref import synthetic_inat_names
    from oracle.swinv2_ref import init_params_from_rng
    if "modules" not in only:
        return main_models(ref, ref_h, only)
    # ---------------------------------------------------------------- modules
    mods = {}

    def set_params(m, seed):
        shapes = {k: v.shape for k, v in m.state_dict().items()
                  if v.dtype.is_floating_point and not k.endswith("logit_clamp_max")
                  and "relative_coords_table" not in k and "attn_mask" not in k}
        p = init_params_from_rng(shapes, seed)
        m.load_state_dict(p, strict=False)
        return p

    def run(m, prefix, x, seed, mask=None):
        m.zero_grad(set_to_none=True)  # wattn_* run the same module twice
        x = x.clone().requires_grad_(True)
        y = m(x) if mask is None else m(x, mask=mask)
        g = torch.from_numpy(np.random.default_rng(seed + 1).standard_normal(
            tuple(y.shape)).astype(np.float32))
        y.backward(g)
        mods[prefix + "x"] = x.detach().numpy()
        mods[prefix + "y"] = y.detach().numpy()
        mods[prefix + "gy"] = g.numpy()
        mods[prefix + "gx"] = x.grad.numpy().copy()
        for k, v in m.named_parameters():
            if v.grad is not None:
                mods[prefix + "grad." + k] = v.grad.numpy().copy()  # the module may run again

    rng = np.random.default_rng(1234)
    # WindowAttention with a shift mask: dim 64, 2 heads (head_dim 32), w 7, res 14
    blk = ref.SwinTransformerBlock(dim=64, input_resolution=(14, 14), num_heads=2,
                                   window_size=7, shift_size=3)
    wa = blk.attn
    set_params(wa, 11)
    xw = torch.from_numpy(rng.standard_normal((2 * 4, 49, 64)).astype(np.float32))
    run(wa, "wattn_mask.", xw, 12, mask=blk.attn_mask)
    set_params(wa, 13)
    run(wa, "wattn_nomask.", xw, 14)
    for s in (0, 3):
        blk = ref.SwinTransformerBlock(dim=64, input_resolution=(14, 14), num_heads=2,
                                       window_size=7, shift_size=s)
        set_params(blk, 20 + s)
        x = torch.from_numpy(rng.standard_normal((2, 196, 64)).astype(np.float32))
        run(blk, f"block_s{s}.", x, 30 + s)
    # 16x16 map, window 8 (N = 64), shifted
    blk = ref.SwinTransformerBlock(dim=64, input_resolution=(16, 16), num_heads=2,
                                   window_size=8, shift_size=4)
    set_params(blk, 40)
    x = torch.from_numpy(rng.standard_normal((2, 256, 64)).astype(np.float32))
    run(blk, "block_w8s4.", x, 41)
    pm = ref.PatchMerging((14, 14), dim=32)
    set_params(pm, 50)
    x = torch.from_numpy(rng.standard_normal((2, 196, 32)).astype(np.float32))
    run(pm, "merge.", x, 51)
    mlp = ref.Mlp(in_features=32, hidden_features=128)
    set_params(mlp, 60)
    x = torch.from_numpy(rng.standard_normal((3, 5, 32)).astype(np.float32))
    run(mlp, "mlp.", x, 61)
    np.savez_compressed(os.path.join(HERE, "module_golden.npz"), **mods)
    main_models(ref, ref_h, only)


def main_models(ref, ref_h, only):
    from oracle.hierarchy_ref import synthetic_inat_names
    from oracle.swinv2_ref import init_params_from_rng
    if "models" not in only:
        return main_tax(ref, ref_h, only)
    # ---------------------------------------------------------------- models
    models = {}
    cfgs = {
        # tiny config for fast tests: stage0 res 14 (shifted 2x2 windows), stage1 7x7
        "mini": dict(img_size=56, embed_dim=32, depths=[2, 2], num_heads=[1, 2],
                     window_size=7, num_classes=10, drop_path_rate=0.0),
        "mini_mt": dict(img_size=56, embed_dim=32, depths=[2, 2], num_heads=[1, 2],
                        window_size=7, num_classes=(3, 4, 5, 6, 7, 8, 9),
                        drop_path_rate=0.0),
        "tiny": dict(img_size=224, embed_dim=96, depths=[2, 2, 6, 2],
                     num_heads=[3, 6, 12, 24], window_size=7, num_classes=1000,
                     drop_path_rate=0.0),
    }
    for name, cfg in cfgs.items():
        net = ref.SwinTransformerV2(**cfg).eval()
        shapes = {k: v.shape for k, v in net.state_dict().items()
                  if k.endswith(("weight", "bias", "logit_scale"))
                  and "relative" not in k}
        p = init_params_from_rng(shapes, 7)
        missing, unexpected = net.load_state_dict(p, strict=False)
        assert not unexpected, unexpected
        b = 2
        x = torch.from_numpy(np.random.default_rng(42).standard_normal(
            (b, 3, cfg["img_size"], cfg["img_size"])).astype(np.float32))
        with torch.no_grad():
            y = net(x)
            with torch.autocast("cpu", dtype=torch.bfloat16):
                yb = net(x)
        if isinstance(y, list):
            for i, (a, c) in enumerate(zip(y, yb)):
                models[f"{name}.logits{i}"] = a.numpy()
                models[f"{name}.logits_bf16_{i}"] = c.float().numpy()
        else:
            models[f"{name}.logits"] = y.numpy()
            models[f"{name}.logits_bf16"] = yb.float().numpy()
        models[f"{name}.n_state_keys"] = np.array(len(net.state_dict()))
        models[f"{name}.macs"] = np.array(net.flops(), np.float64)
        if name == "mini":
            # one backward for the parameter-gradient parity test
            net.train()
            xx = x.clone().requires_grad_(True)
            out = net(xx)
            g = torch.from_numpy(np.random.default_rng(43).standard_normal(
                tuple(out.shape)).astype(np.float32))
            out.backward(g)
            models["mini.gx"] = xx.grad.numpy()
            for k, v in net.named_parameters():
                models["mini.grad." + k] = v.grad.numpy()
            # the same backward under CPU bf16 autocast: the reference's own bf16 error
            net.zero_grad()
            xx = x.clone().requires_grad_(True)
            with torch.autocast("cpu", dtype=torch.bfloat16):
                out = net(xx)
            out.float().backward(g)
            models["mini.gx_bf16"] = xx.grad.float().numpy()
            for k, v in net.named_parameters():
                models["mini.grad_bf16." + k] = v.grad.float().numpy()
    keys = list(ref.SwinTransformerV2(**cfgs["tiny"]).state_dict().keys())
    models["tiny.state_keys"] = np.array(keys)
    np.savez_compressed(os.path.join(HERE, "model_golden.npz"), **models)
    main_tax(ref, ref_h, only)


def main_tax(ref, ref_h, only):
    from oracle.hierarchy_ref import synthetic_inat_names
    if "taxonomy" not in only:
        return main_loss(ref, ref_h, only)
    # ---------------------------------------------------------------- taxonomy
    tax = {}
    names = synthetic_inat_names()
    rng = np.random.default_rng(5)
    shuffled = list(rng.permutation(np.array(names)))
    classes, c2i = ref_h.HierarchicalImageFolder.find_classes(
        types.SimpleNamespace(), _FakeDir(shuffled))
    tax["synthetic.classes"] = np.array(classes)
    tax["synthetic.ids"] = np.stack([c2i[c].numpy() for c in classes]).astype(np.int64)
    nc = tuple(int(tax["synthetic.ids"][:, t].max()) + 1 for t in range(7))
    tax["synthetic.num_classes"] = np.array(nc)
    hand = ["00001_animalia_chordata_aves_accipitriformes_accipitridae_haliaeetus_leucocephalus",
            "00002_animalia_chordata_reptilia_accipitriformes_accipitridae_haliaeetus_leucocephalus",
            "00000_plantae_tracheophyta_magnoliopsida_rosales_rosaceae_rosa_canina",
            "00003_plantae_tracheophyta_magnoliopsida_rosales_rosaceae_rosa_rugosa",
            "00004_fungi_basidiomycota_agaricomycetes_agaricales_amanitaceae_amanita_muscaria"]
    classes, c2i = ref_h.HierarchicalImageFolder.find_classes(
        types.SimpleNamespace(), _FakeDir(hand))
    tax["hand.classes"] = np.array(classes)
    tax["hand.ids"] = np.stack([c2i[c].numpy() for c in classes]).astype(np.int64)
    tax["hand.tiers"] = np.array([ref_h.HierarchicalLabel.parse(c).clean_tiers for c in classes])
    labels = [ref_h.HierarchicalLabel.parse(c) for c in classes]
    tax["hand.dist"] = np.array([[a.dist(b) for b in labels] for a in labels], np.int64)
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        for split in ("train", "val"):
            os.makedirs(os.path.join(d, split))
        sub = names[:: 97]
        for i, n in enumerate(sub):
            os.makedirs(os.path.join(d, "train" if i % 3 else "val", n))
        vecs = ref_h.build_parent_label_lookup(d)
        tax["parent.names"] = np.array(sub)
        for i, v in enumerate(vecs):
            tax[f"parent.vec{i}"] = v
    np.savez_compressed(os.path.join(HERE, "taxonomy_golden.npz"), **tax)
    main_loss(ref, ref_h, only)


def main_loss(ref, ref_h, only):
    if "losses" not in only:
        return
    # ---------------------------------------------------------------- losses
    loss = {}
    sizes = (3, 13, 51, 273, 1103, 4884, 10000)
    coeffs = [8, 5.65, 4, 2.82, 2, 1.41, 1]
    rng = np.random.default_rng(77)
    b = 4
    logits = [torch.from_numpy((2.0 * rng.standard_normal((b, n))).astype(np.float32))
              for n in sizes]
    targets = torch.from_numpy(np.stack([rng.integers(0, n, b) for n in sizes], 1))
    fn = ref_h.MultitaskCrossEntropy(coeffs=coeffs)
    lh = fn(logits, targets)
    eps = 0.08
    soft = [torch.nn.functional.one_hot(t, n).float() * (1 - eps) + eps / n
            for t, n in zip(targets.T, sizes)]
    ls = fn(logits, soft)
    for i, z in enumerate(logits):
        loss[f"mt.logits{i}"] = z.numpy()
    loss["mt.targets"] = targets.numpy()
    loss["mt.coeffs"] = np.array(coeffs, np.float32)
    loss["mt.loss_hard"] = np.array(float(lh))
    loss["mt.loss_soft"] = np.array(float(ls))
    loss["mt.smoothing"] = np.array(eps)
    np.savez_compressed(os.path.join(HERE, "loss_golden.npz"), **loss)
    print("goldens written to", HERE)


PROD_BLOCKS = {
    # SwinV2-T stage 0 (56x56, C 96, 3 heads, shifted) and stage 2 (14x14, C 384, 12 heads),
    # SwinV2-B stage 0 width (C 128, 4 heads) on a 14x14 shifted map
    "t_s0": dict(dim=96, res=56, heads=3, window=7, shift=3, batch=1, seed=100),
    "t_s2": dict(dim=384, res=14, heads=12, window=7, shift=3, batch=2, seed=110),
    "b_s0": dict(dim=128, res=14, heads=4, window=7, shift=3, batch=2, seed=120),
}
SWINB = {
    # BASELINE configs[3] / [4] geometries (models.py registry names; swinv2.py:699-719)
    "b224_mt": dict(img_size=224, embed_dim=128, depths=[2, 2, 18, 2], num_heads=[4, 8, 16, 32],
                    window_size=7, num_classes=(3, 13, 51, 273, 1103, 4884, 10000),
                    drop_path_rate=0.0),
    "b384_w24": dict(img_size=384, embed_dim=128, depths=[2, 2, 18, 2], num_heads=[4, 8, 16, 32],
                     window_size=24, pretrained_window_sizes=[12, 12, 12, 6], num_classes=10000,
                     drop_path_rate=0.0),
}


def swinb_and_prod(ref, init_params_from_rng, which):
    """prod_golden.npz: production-width SwinTransformerBlocks (random post-norm gammas) with
    sampled outputs, input gradients and every parameter gradient; swinb_golden.npz: SwinV2-B
    224 multitask and 384 w24 logits (B = 1), f32 and CPU bf16 autocast."""
    out = {}
    if which == "prod":
        for name, c in PROD_BLOCKS.items():
            blk = ref.SwinTransformerBlock(dim=c["dim"], input_resolution=(c["res"], c["res"]),
                                           num_heads=c["heads"], window_size=c["window"],
                                           shift_size=c["shift"])
            shapes = {k: v.shape for k, v in blk.state_dict().items()
                      if v.dtype.is_floating_point and not k.endswith("logit_clamp_max")
                      and "relative_coords_table" not in k and "attn_mask" not in k}
            blk.load_state_dict(init_params_from_rng(shapes, c["seed"]), strict=False)
            L = c["res"] * c["res"]
            x = torch.from_numpy(seeded(c["seed"] + 1, (c["batch"], L, c["dim"]))).requires_grad_(True)
            y = blk(x)
            gy = torch.from_numpy(seeded(c["seed"] + 2, tuple(y.shape)))
            y.backward(gy)
            pre = name + "."
            out[pre + "y"] = sampled(pre + "y", y.detach().numpy())
            out[pre + "gx"] = sampled(pre + "gx", x.grad.numpy())
            for k, v in blk.named_parameters():
                out[pre + "grad." + k] = sampled(pre + "grad." + k, v.grad.numpy())
        np.savez_compressed(os.path.join(HERE, "prod_golden.npz"), **out)
        return
    for name, cfg in SWINB.items():
        net = ref.SwinTransformerV2(**cfg).eval()
        shapes = {k: v.shape for k, v in net.state_dict().items()
                  if k.endswith(("weight", "bias", "logit_scale")) and "relative" not in k}
        missing, unexpected = net.load_state_dict(init_params_from_rng(shapes, 7), strict=False)
        assert not unexpected, unexpected
        x = torch.from_numpy(seeded(42, (1, 3, cfg["img_size"], cfg["img_size"])))
        with torch.no_grad():
            y = net(x)
            with torch.autocast("cpu", dtype=torch.bfloat16):
                yb = net(x)
        ys, ybs = (y, yb) if isinstance(y, list) else ([y], [yb])
        for i, (a, b) in enumerate(zip(ys, ybs)):
            out[f"{name}.logits{i}"] = a.numpy()
            out[f"{name}.logits_bf16_{i}"] = b.float().numpy()
        out[f"{name}.n_state_keys"] = np.array(len(net.state_dict()))
        out[f"{name}.macs"] = np.array(net.flops(), np.float64)
    np.savez_compressed(os.path.join(HERE, "swinb_golden.npz"), **out)


STEPS = {
    # whole training steps (loss + every parameter gradient) of BASELINE configs[2..4]:
    # (model cfg, batch, loss); drop_path 0 (the shim's DropPath is the identity)
    "t_hxe": (dict(img_size=224, embed_dim=96, depths=[2, 2, 6, 2], num_heads=[3, 6, 12, 24],
                   window_size=7, num_classes=10000, drop_path_rate=0.0), 2, "hxe"),
    "b224_mt": (SWINB["b224_mt"], 1, "multitask"),
    "b384_hxe": (SWINB["b384_w24"], 1, "hxe"),
}
STEP_SAMPLES = 512
MT_COEFFS = [8, 5.65, 4, 2.82, 2, 1.41, 1]  # configs/pretrain/r50_multitask_base.yaml:3


def train_steps(ref, ref_h, init_params_from_rng):
    """step_golden.npz: per config, the reference network's loss and parameter gradients for one
    step, in f32 and under CPU bf16 autocast (the reference's own bf16 error: the tests bound
    the HIP path by max(base, 1.5 x that error) per tensor).  Multitask: the reference's
    MultitaskCrossEntropy (hierarchy.py:65-94).  HXE: not implemented by the reference
    (hierarchy.py:183-185), so the loss on the reference's logits is the oracle's HXE
    (hierarchy_ref.hxe_loss_torch, pinned by closed-form tests) -- the network half is the
    reference's.  Gradients are stored sampled (STEP_SAMPLES entries, tests/golden_util.py);
    the bf16 error is measured on the full tensors and stored as one number per tensor."""
    sys.path.insert(0, REPO)
    from oracle import hierarchy_ref
    from hvamd.hierarchy import Taxonomy
    tax = Taxonomy.synthetic()
    lam = hierarchy_ref.hxe_level_weights("exponential", 0.1)
    out = {}
    for name, (cfg, B, loss_kind) in STEPS.items():
        net = ref.SwinTransformerV2(**cfg).train()
        shapes = {k: v.shape for k, v in net.state_dict().items()
                  if k.endswith(("weight", "bias", "logit_scale")) and "relative" not in k}
        missing, unexpected = net.load_state_dict(init_params_from_rng(shapes, 7), strict=False)
        assert not unexpected, unexpected
        x = torch.from_numpy(seeded(42, (B, 3, cfg["img_size"], cfg["img_size"])))
        leaves = np.random.default_rng(43).integers(0, tax.num_leaves, B)
        paths = tax.leaf_paths[leaves]
        out[f"{name}.leaves"] = leaves

        def loss_of(z):
            if loss_kind == "hxe":
                return hierarchy_ref.hxe_loss_torch(z.float(), paths, tax.perm, tax.node_start,
                                                    tax.node_end, tax.tier_base, lam)
            return ref_h.MultitaskCrossEntropy(coeffs=MT_COEFFS)([t.float() for t in z],
                                                                 torch.from_numpy(paths))
        grads = {}
        for prec in ("f32", "bf16"):
            net.zero_grad()
            with torch.autocast("cpu", dtype=torch.bfloat16, enabled=prec == "bf16"):
                z = net(x)
            loss = loss_of(z)
            loss.backward()
            out[f"{name}.loss_{prec}"] = np.array(float(loss))
            grads[prec] = {k: v.grad.detach().float().clone() for k, v in net.named_parameters()
                           if v.grad is not None}
            print(name, prec, float(loss), flush=True)
        for k, g32 in grads["f32"].items():
            g16 = grads["bf16"][k]
            out[f"{name}.g.{k}"] = sampled(f"{name}.g.{k}", g32.numpy(), STEP_SAMPLES)
            out[f"{name}.e16.{k}"] = np.array(float((g16 - g32).norm() / g32.norm().clamp_min(1e-30)))
        del net, grads
    np.savez_compressed(os.path.join(HERE, "step_golden.npz"), **out)


BENCH_BLOCKS = {
    # SwinV2-T stages 1-3 at the batch sizes where the product takes its bench routing
    # (hvamd/ops.py _tile_ok: the tiled GEMMs from M >= 32768 tokens at stages 1-2, M >= 8192 at
    # stage 3, the stage-1 norm in the 128 x 192 tile's epilogue, the qkv normalisation epilogue)
    "t_s1_b48": dict(dim=192, res=28, heads=6, window=7, shift=3, batch=48, seed=130),
    "t_s2_b168": dict(dim=384, res=14, heads=12, window=7, shift=3, batch=168, seed=140),
    "t_s3_b192": dict(dim=768, res=7, heads=24, window=7, shift=0, batch=192, seed=150),
    # a ragged token count (M = 176 x 49, not a multiple of the weight-gradient kernel's 32-token
    # stage): the dW launches split into an aligned part and a zero-padded tail
    "t_s3_b176": dict(dim=768, res=7, heads=24, window=7, shift=0, batch=176, seed=155),
}
BENCH_MERGES = {
    # the three SwinV2-T PatchMergings at the same sizes (gather folded into the reduction GEMM;
    # the stage-0 -> 1 one with its norm in the tile epilogue)
    "m01_b48": dict(dim=96, res=56, batch=48, seed=160),
    "m12_b168": dict(dim=192, res=28, batch=168, seed=170),
    "m23_b192": dict(dim=384, res=14, batch=192, seed=180),
    "m23_b176": dict(dim=384, res=14, batch=176, seed=185),  # ragged: gather + tile GEMM, split dW
}


def bench_batch_modules(ref, init_params_from_rng):
    """prodb_golden.npz: BENCH_BLOCKS / BENCH_MERGES in f32 (sampled output, input gradient and
    every parameter gradient) plus the reference's own CPU bf16-autocast error per tensor
    (relative L2 over the full tensor), from which the tests derive their bounds."""
    out = {}
    mods = [(n, c, "block") for n, c in BENCH_BLOCKS.items()] + [(n, c, "merge") for n, c in BENCH_MERGES.items()]
    for name, c, kind in mods:
        if kind == "block":
            m = ref.SwinTransformerBlock(dim=c["dim"], input_resolution=(c["res"], c["res"]), num_heads=c["heads"],
                                         window_size=c["window"], shift_size=c["shift"])
        else:
            m = ref.PatchMerging((c["res"], c["res"]), dim=c["dim"])
        shapes = {k: v.shape for k, v in m.state_dict().items()
                  if v.dtype.is_floating_point and not k.endswith("logit_clamp_max")
                  and "relative_coords_table" not in k and "attn_mask" not in k}
        m.load_state_dict(init_params_from_rng(shapes, c["seed"]), strict=False)
        L = c["res"] * c["res"]
        xin = torch.from_numpy(seeded(c["seed"] + 1, (c["batch"], L, c["dim"])))
        res = {}
        for prec in ("f32", "bf16"):
            m.zero_grad(set_to_none=True)
            x = xin.clone().requires_grad_(True)
            with torch.autocast("cpu", dtype=torch.bfloat16, enabled=prec == "bf16"):
                y = m(x)
            gy = torch.from_numpy(seeded(c["seed"] + 2, tuple(y.shape)))
            y.float().backward(gy)
            res[prec] = {"y": y.detach().float(), "gx": x.grad.float()}
            res[prec].update({"grad." + k: v.grad.detach().float().clone() for k, v in m.named_parameters()})
        pre = name + "."
        for k, a in res["f32"].items():
            out[pre + k] = sampled(pre + k, a.numpy())
            out[pre + "e16." + k] = np.array(float((res["bf16"][k] - a).norm() / a.norm().clamp_min(1e-30)))
        print(name, {k: round(float(out[pre + "e16." + k]), 4) for k in res["f32"]}, flush=True)
    np.savez_compressed(os.path.join(HERE, "prodb_golden.npz"), **out)


STEP256 = dict(img_size=224, embed_dim=96, depths=[2, 2, 6, 2], num_heads=[3, 6, 12, 24], window_size=7,
               num_classes=10000, drop_path_rate=0.0)
STEP256_BATCH, STEP256_CHUNK = 256, 32


def train_step_b256(ref, init_params_from_rng):
    """step256_golden.npz: the bench's own step (BASELINE configs[2]: SwinV2-T 224 + HXE over the
    10 000-leaf tree, batch 256) on the reference network, f32 and CPU bf16 autocast: loss and
    every parameter gradient (sampled) plus the reference's own bf16 error per tensor.  The batch
    runs as 8 chunks of 32 with each chunk's loss scaled by 32/256 and the gradients accumulated
    (the same sum as one batch of 256, in 8 pieces, so the reference's CPU activations fit this
    container's memory).  HXE is the oracle's (hierarchy.py:183-185 raises), as in train_steps."""
    sys.path.insert(0, REPO)
    from oracle import hierarchy_ref
    from hvamd.hierarchy import Taxonomy
    tax = Taxonomy.synthetic()
    lam = hierarchy_ref.hxe_level_weights("exponential", 0.1)
    net = ref.SwinTransformerV2(**STEP256).train()
    shapes = {k: v.shape for k, v in net.state_dict().items()
              if k.endswith(("weight", "bias", "logit_scale")) and "relative" not in k}
    missing, unexpected = net.load_state_dict(init_params_from_rng(shapes, 7), strict=False)
    assert not unexpected, unexpected
    B, CH = STEP256_BATCH, STEP256_CHUNK
    x = seeded(42, (B, 3, 224, 224))
    leaves = np.random.default_rng(43).integers(0, tax.num_leaves, B)
    paths = tax.leaf_paths[leaves]
    out = {"t256.leaves": leaves, "t256.x_checksum": np.array([float(x.astype(np.float64).sum()),
                                                               float(np.abs(x).astype(np.float64).sum())])}
    grads = {}
    for prec in ("f32", "bf16"):
        net.zero_grad(set_to_none=True)
        total = 0.0
        for c0 in range(0, B, CH):
            with torch.autocast("cpu", dtype=torch.bfloat16, enabled=prec == "bf16"):
                z = net(torch.from_numpy(x[c0:c0 + CH]))
            loss = hierarchy_ref.hxe_loss_torch(z.float(), paths[c0:c0 + CH], tax.perm, tax.node_start,
                                                tax.node_end, tax.tier_base, lam) * (CH / B)
            loss.backward()
            total += float(loss)
            print("t256", prec, c0, float(loss), flush=True)
        out[f"t256.loss_{prec}"] = np.array(total)
        grads[prec] = {k: v.grad.detach().float().clone() for k, v in net.named_parameters() if v.grad is not None}
    for k, g32 in grads["f32"].items():
        out[f"t256.g.{k}"] = sampled(f"t256.g.{k}", g32.numpy(), STEP_SAMPLES)
        out[f"t256.e16.{k}"] = np.array(float((grads["bf16"][k] - g32).norm() / g32.norm().clamp_min(1e-30)))
    np.savez_compressed(os.path.join(HERE, "step256_golden.npz"), **out)


class _FakeDir(str):
    """find_classes() scans a directory; hand it names through os.scandir."""

    def __new__(cls, names):
        s = super().__new__(cls, "<fake>")
        s.names = list(names)
        return s


_real_scandir = os.scandir


def _scandir(path="."):
    if isinstance(path, _FakeDir):
        return iter([types.SimpleNamespace(name=n, is_dir=lambda: True) for n in path.names])
    return _real_scandir(path)


os.scandir = _scandir

if __name__ == "__main__":
    main()
