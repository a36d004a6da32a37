"""Model / loss boundary -- drop-in for models.py.

``build_model(config, num_classes)`` resolves ``config.model.name`` through a
SwinV2 registry (the reference calls timm.create_model, models.py:19/25, which
is absent offline; the registry gives the official SwinV2 geometries with the
semantics of swinv2.py).  ``build_composer_model`` picks the loss by
``config.hierarchy.variant`` in {"", "multitask", "hxe"} (models.py:105-114;
"hxe" is implemented here, the reference raises).  ``Model`` keeps the
ComposerModel method surface: forward(batch), loss(outputs, batch),
get_metrics(is_train), update_metric(batch, outputs, metric).
"""
import dataclasses

import torch

from . import hierarchy
from .swinv2 import SwinTransformerV2

# name -> SwinTransformerV2 kwargs (official SwinV2 configs; drop_path 0.1 = swinv2.py:713 default)
MODEL_REGISTRY = {
    "swinv2_tiny_window7_224": dict(img_size=224, embed_dim=96, depths=[2, 2, 6, 2],
                                    num_heads=[3, 6, 12, 24], window_size=7),
    "swinv2_small_window7_224": dict(img_size=224, embed_dim=96, depths=[2, 2, 18, 2],
                                     num_heads=[3, 6, 12, 24], window_size=7),
    "swinv2_base_window7_224": dict(img_size=224, embed_dim=128, depths=[2, 2, 18, 2],
                                    num_heads=[4, 8, 16, 32], window_size=7),
    "swinv2_tiny_window8_256": dict(img_size=256, embed_dim=96, depths=[2, 2, 6, 2],
                                    num_heads=[3, 6, 12, 24], window_size=8),
    "swinv2_small_window8_256": dict(img_size=256, embed_dim=96, depths=[2, 2, 18, 2],
                                     num_heads=[3, 6, 12, 24], window_size=8),
    "swinv2_base_window8_256": dict(img_size=256, embed_dim=128, depths=[2, 2, 18, 2],
                                    num_heads=[4, 8, 16, 32], window_size=8),
    "swinv2_base_window24_384": dict(img_size=384, embed_dim=128, depths=[2, 2, 18, 2],
                                     num_heads=[4, 8, 16, 32], window_size=24,
                                     pretrained_window_sizes=[12, 12, 12, 6]),
}


def create_model(name, num_classes=1000, **kwargs):
    if name not in MODEL_REGISTRY:
        raise ValueError(f"model '{name}' is not provided: this framework implements the SwinV2 "
                         f"hot path only ({', '.join(sorted(MODEL_REGISTRY))})")
    cfg = dict(MODEL_REGISTRY[name])
    cfg.update(kwargs)
    return SwinTransformerV2(num_classes=num_classes, **cfg)


def weight_init(w: torch.nn.Module):
    """Kaiming-normal on every Linear / Conv2d, applied after construction
    (models.py:208-213) -- it overrides swinv2's trunc-normal init."""
    if isinstance(w, (torch.nn.Linear, torch.nn.Conv2d)):
        torch.nn.init.kaiming_normal_(w.weight)


class FeatureOnlyModel(torch.nn.Module):
    """Frozen backbone returning pooled features (models.py:186-205)."""

    def __init__(self, backbone):
        super().__init__()
        self.backbone = backbone
        self.backbone.eval()
        self.backbone.requires_grad_(False)

    def forward(self, x):
        self.backbone.eval()
        return self.backbone.forward_head(self.backbone.forward_features(x), pre_logits=True)


def build_model(config, num_classes, **model_kwargs):
    """models.py:16-51."""
    if isinstance(num_classes, int):
        model = create_model(config.model.name, num_classes=num_classes, **model_kwargs)
    elif isinstance(num_classes, tuple):
        assert config.hierarchy.variant == "multitask", \
            "config.hierarchy.variant must be multitask to use with multiple tiers of classes!"
        model = create_model(config.model.name, num_classes=2, **model_kwargs)
        if hasattr(model, "fc"):
            hierarchy.multitask_surgery(model, "fc", num_classes)
        elif hasattr(model, "head"):
            hierarchy.multitask_surgery(model, "head", num_classes)
        else:
            raise NotImplementedError("don't how to apply hierarchical multitask head to model!")
    else:
        raise TypeError(f"num_classes must be int or (int, int ...), not {type(num_classes)}")
    model.apply(weight_init)
    if config.model.variant == "full-tuning":
        pass
    elif config.model.variant in ("linear-probe", "simpleshot", "simpleshot-l2n", "simpleshot-cl2n"):
        model = FeatureOnlyModel(model)
    else:
        raise ValueError(config.model.variant)
    return model


@dataclasses.dataclass(frozen=True)
class DatasetInfo:
    """data.py:79-90 plus the taxonomy HXE needs."""
    num_classes: object
    tree_dists: object = None
    taxonomy: object = None


class Model(torch.nn.Module):
    """ComposerModel surface (models.py:121-152)."""

    def __init__(self, module, train_metrics, val_metrics, loss_fn):
        super().__init__()
        self.module = module
        self.loss_fn = loss_fn
        self.train_metrics = train_metrics
        self.val_metrics = val_metrics

    def loss(self, outputs, batch, *args, **kwargs):
        _, targets = batch
        return self.loss_fn(outputs, targets, *args, **kwargs)

    def get_metrics(self, is_train=False):
        return self.train_metrics if is_train else self.val_metrics

    def update_metric(self, batch, outputs, metric):
        _, targets = batch
        metric.update(outputs, targets)

    def forward(self, batch):
        inputs, _ = batch
        return self.module(inputs)


def build_composer_model(config, dataset_info: DatasetInfo, **model_kwargs):
    """models.py:54-118 with the "hxe" branch implemented."""
    variant = config.hierarchy.variant
    num_classes = dataset_info.num_classes
    if variant == "hxe":
        tax = dataset_info.taxonomy
        if tax is None:
            raise ValueError("hierarchy.variant=hxe needs DatasetInfo.taxonomy")
        num_classes = tax.num_leaves
    model = build_model(config, num_classes, **model_kwargs)

    # metrics (models.py:61-101): the same dict keys per variant; "hxe" scores its leaf
    # logits as the flat variant does
    if variant == "multitask":
        def fine_grained():
            return {"cross-entropy": hierarchy.FineGrainedCrossEntropy(),
                    "acc@1": hierarchy.FineGrainedAccuracy(topk=1),
                    "acc@5": hierarchy.FineGrainedAccuracy(topk=5)}
        train_metrics = fine_grained()
        val_metrics = fine_grained()
        val_metrics["tree-dist"] = hierarchy.FineGrainedTreeDistance(dataset_info.tree_dists)
        if not config.is_train:
            train_metrics["tree-dist"] = hierarchy.FineGrainedTreeDistance(dataset_info.tree_dists)
            val_metrics["tree-dist"] = hierarchy.FineGrainedTreeDistance(dataset_info.tree_dists)
    else:
        assert isinstance(num_classes, int)

        def flat():
            return {"cross-entropy": hierarchy.CrossEntropyMetric(),
                    "acc@1": hierarchy.Accuracy(num_classes=num_classes),
                    "acc@5": hierarchy.Accuracy(num_classes=num_classes, top_k=5)}
        train_metrics = flat()
        val_metrics = flat()
        if not config.is_train:
            train_metrics["tree-dist"] = hierarchy.TreeDistance(dataset_info.tree_dists)
            val_metrics["tree-dist"] = hierarchy.TreeDistance(dataset_info.tree_dists)

    if variant == "hxe":
        loss_fn = hierarchy.HierarchicalCrossEntropy(dataset_info.taxonomy,
                                                     tree_weights=config.hierarchy.hxe_tree_weights,
                                                     alpha=config.hierarchy.hxe_alpha)
    elif variant == "multitask":
        loss_fn = hierarchy.MultitaskCrossEntropy(coeffs=config.hierarchy.multitask_coeffs)
    elif variant == "":
        loss_fn = hierarchy.soft_cross_entropy
    else:
        raise ValueError(variant)
    return Model(model, train_metrics=train_metrics, val_metrics=val_metrics, loss_fn=loss_fn)
