"""Composer-style algorithms that touch the hot path (algorithmic.py).

Minimal Event / State / Algorithm surface (match(event, state) / apply(event,
state, logger)) so the reference's `algorithms:` YAML entries drive this
trainer the way they drive composer.Trainer (main.py:98-102).
"""
import dataclasses
import enum
import logging
import math
import os
import re

import torch

log = logging.getLogger(__name__)


class Event(enum.Enum):
    INIT = "init"
    BATCH_START = "batch_start"
    BEFORE_FORWARD = "before_forward"
    AFTER_FORWARD = "after_forward"
    BEFORE_LOSS = "before_loss"
    AFTER_LOSS = "after_loss"
    BEFORE_BACKWARD = "before_backward"
    AFTER_BACKWARD = "after_backward"
    BATCH_END = "batch_end"


class State:
    """The slice of composer.State the algorithms use."""

    def __init__(self, model, optimizer=None):
        self.model = model
        self.optimizers = [optimizer] if optimizer is not None else []
        self.batch = None
        self.outputs = None
        self.loss = None
        self.timestamp_batch = 0

    def batch_get_item(self, key):
        return self.batch[key]

    def batch_set_item(self, key, value):
        b = list(self.batch)
        b[key] = value
        self.batch = tuple(b)


class Algorithm:
    def match(self, event, state) -> bool:
        raise NotImplementedError

    def apply(self, event, state, logger=None):
        raise NotImplementedError


def smooth_labels(logits: torch.Tensor, target: torch.Tensor, smoothing: float = 0.1):
    """(one_hot(target) * (1 - smoothing)) + smoothing / n_classes (algorithmic.py:160-164)."""
    n_classes = logits.shape[1]
    if target.dtype.is_floating_point and target.shape == logits.shape:
        one_hot = target
    else:
        one_hot = torch.nn.functional.one_hot(target.long(), n_classes).to(logits.dtype)
    return (one_hot.float() * (1.0 - smoothing)) + (smoothing / n_classes)


class LabelSmoothing(Algorithm):
    """Label smoothing that also handles multitask list outputs (algorithmic.py:88-119):
    BEFORE_LOSS swaps the targets for smoothed probability targets (one per tier
    for list outputs); AFTER_LOSS restores the originals."""

    def __init__(self, smoothing=0.1, target_key=1):
        self.smoothing = smoothing
        self.target_key = target_key
        self.original_labels = None

    def match(self, event, state):
        return event in (Event.BEFORE_LOSS, Event.AFTER_LOSS)

    def apply(self, event, state, logger=None):
        if event == Event.BEFORE_LOSS:
            labels = state.batch_get_item(self.target_key)
            assert isinstance(labels, torch.Tensor), "type error"
            self.original_labels = labels.clone()
            if isinstance(state.outputs, list):
                b, tiers = labels.shape
                assert len(state.outputs) == tiers, "different level of tiers"
                assert all(o.shape[0] == b for o in state.outputs), "different batch sizes"
                smoothed = [smooth_labels(o, t, self.smoothing) for o, t in zip(state.outputs, labels.T)]
            else:
                smoothed = smooth_labels(state.outputs, labels, self.smoothing)
            state.batch_set_item(self.target_key, smoothed)
        elif event == Event.AFTER_LOSS:
            state.batch_set_item(self.target_key, self.original_labels)


class GradientClipping(Algorithm):
    """Global-norm (or value) clipping after backward (configs/pretrain/inat21.yaml:44-47)."""

    def __init__(self, clipping_type="norm", clipping_threshold=2.0):
        if clipping_type not in ("norm", "value"):
            raise ValueError(clipping_type)
        self.clipping_type = clipping_type
        self.clipping_threshold = clipping_threshold

    def match(self, event, state):
        return event == Event.AFTER_BACKWARD

    def apply(self, event, state, logger=None):
        params = [p for p in state.model.parameters() if p.grad is not None]
        opts = getattr(state, "optimizers", None) or []
        opt = opts[0] if len(opts) == 1 else None
        if (self.clipping_type == "norm" and opt is not None
                and getattr(opt, "supports_fused_clip", lambda: False)()
                and {id(p) for p in params} <= {id(q) for g in opt.param_groups for q in g["params"]}):
            # the optimizer's step applies the clip coefficient on the fly (same global norm,
            # computed on the device in the fused update, no host synchronisation)
            opt.pending_clip = self.clipping_threshold
            return
        # clipping here, not in the optimizer: a DDP mean still pending as the optimizer's
        # gradient scale (trainer._grad_mean hands 1/world over) must be applied first, or the
        # threshold would act on world-times gradients
        for o in opts:
            scale = getattr(o, "pending_grad_scale", 1.0)
            if scale != 1.0:
                mine = [q.grad for g in o.param_groups for q in g["params"] if q.grad is not None]
                if mine:
                    torch._foreach_mul_(mine, float(scale))
                o.pending_grad_scale = 1.0
        if self.clipping_type == "norm":
            torch.nn.utils.clip_grad_norm_(params, self.clipping_threshold, foreach=True)
        else:
            torch.nn.utils.clip_grad_value_(params, self.clipping_threshold, foreach=True)


class EMA(Algorithm):
    """Exponential moving average of the weights every `update_interval` batches with
    smoothing from a half-life in batches (configs/pretrain/inat21.yaml:32-35).

    On an update batch the average is handed to an optimizer that can fold it into its own
    pass over the weights (optim.DecoupledSGDW's fused step: ema = a ema + (1 - a) p with the
    freshly updated p, so the weights are not read again); otherwise, and in HIP-graph replays
    (the captured update runs every step), it runs as foreach passes at BATCH_END."""

    def __init__(self, half_life="100ba", update_interval="20ba", smoothing=None):
        hl = int(str(half_life).rstrip("ba"))
        self.update_interval = int(str(update_interval).rstrip("ba"))
        self.smoothing = smoothing if smoothing is not None else math.exp(
            -math.log(2) * self.update_interval / hl)
        self.ema_params = None
        self._handed = False

    def match(self, event, state):
        return event in (Event.AFTER_BACKWARD, Event.BATCH_END)

    @torch.no_grad()
    def apply(self, event, state, logger=None):
        params = [p for p in state.model.parameters()]
        if event == Event.AFTER_BACKWARD:
            self._handed = False
            if self.ema_params is None or (state.timestamp_batch + 1) % self.update_interval:
                return
            if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
                return
            opts = getattr(state, "optimizers", None) or []
            opt = opts[0] if len(opts) == 1 else None
            if (opt is not None and all(p.grad is not None for p in params)
                    and getattr(opt, "supports_fused_ema", lambda ps: False)(params)):
                opt.pending_ema = ([(id(p), e) for p, e in zip(params, self.ema_params)],
                                   self.smoothing)
                self._handed = True
            return
        if self.ema_params is None:
            self.ema_params = [p.detach().clone() for p in params]
            return
        if state.timestamp_batch % self.update_interval:
            return
        if self._handed:  # folded into this step's optimizer pass
            self._handed = False
            return
        torch._foreach_mul_(self.ema_params, self.smoothing)
        torch._foreach_add_(self.ema_params, [p.detach() for p in params], alpha=1 - self.smoothing)


def load_composer_model_dict(path):
    """The model state of a composer checkpoint file: ["state"]["model"] with DDP's "module."
    prefix stripped (algorithmic.py:141-146).  weights_only: nothing in the file executes."""
    model_dict = torch.load(path, map_location="cpu", weights_only=True)["state"]["model"]
    torch.nn.modules.utils.consume_prefix_in_state_dict_if_present(model_dict, "module.")
    return model_dict


@dataclasses.dataclass(frozen=True)
class WandbCheckpoint:
    """`wandb://entity/project/artifact:version?path/in/artifact` (algorithmic.py:120-147).
    The download needs the network; a copy already in the local cache (the reference's own
    cache layout: <cache>/wandb-artifacts/<url>/<filepath>) loads offline."""
    source: str
    url: str
    filepath: str

    @classmethod
    def parse(cls, uri):
        match = re.match(r"^wandb://([\w./-]+:[\w./-]+)\?([\w./-]+)$", uri)
        if not match:
            raise ValueError(f"uri '{uri}' doesn't match the pattern!")
        return cls("wandb", *match.groups())

    def local_path(self, cache):
        return os.path.join(cache, "wandb-artifacts", self.url, self.filepath)

    def load_model_dict(self, cache):
        path = self.local_path(cache)
        if not os.path.exists(path):
            raise RuntimeError(f"W&B artifact {self.url} is not in the local cache ({path}) and "
                               "downloading it needs the network")
        return load_composer_model_dict(path)


def parse_checkpoint(uri: str):
    """algorithmic.py:150-157: a wandb:// or swin:// URI."""
    from .swinv2 import Checkpoint
    for cls in [WandbCheckpoint, Checkpoint]:
        try:
            return cls.parse(uri)
        except ValueError:
            pass
    raise ValueError(f"Could not parse {uri}")


class PretrainedBackbone(Algorithm):
    """Load a pretrained backbone at INIT (algorithmic.py:35-85): the checkpoint's head keys
    are dropped and missing head keys are not reported.  The model's `.backbone` when it has
    one (the linear-probe wrappers), else the network itself.  Accepts wandb:// (offline from
    the local cache) and swin:// URIs (the reference's __init__ parses wandb only)."""

    def __init__(self, checkpoint, local_cache, strict):
        self.checkpoint = parse_checkpoint(checkpoint)
        self.local_cache = local_cache
        self.strict = strict
        os.makedirs(self.local_cache, exist_ok=True)

    def match(self, event, state):
        return event == Event.INIT

    def apply(self, event, state, logger=None):
        module = getattr(state.model, "module", state.model)
        self.load_pretrained_backbone(self.checkpoint, module, self.local_cache, self.strict)

    @staticmethod
    def load_pretrained_backbone(checkpoint, model_with_backbone, local_cache, strict):
        model_dict = checkpoint.load_model_dict(local_cache)
        head_keys = {key for key in model_dict.keys() if "fc." in key or "head." in key}
        for key in head_keys:
            del model_dict[key]
        target = getattr(model_with_backbone, "backbone", model_with_backbone)
        own_head = {k for k in target.state_dict() if "fc." in k or "head." in k}
        missing, unexpected = target.load_state_dict(model_dict, strict=False)
        missing = [k for k in missing if k not in head_keys and k not in own_head
                   and not any(n in k for n in ("relative_position_index", "relative_coords_table",
                                                "logit_clamp_max"))]
        if strict and (missing or unexpected):
            raise RuntimeError(f"pretrained backbone: missing {missing}, unexpected {unexpected}")
        if missing:
            log.warning("Missing keys in checkpoint: %s", ", ".join(missing))
        if unexpected:
            log.warning("Unexpected keys in checkpoint: %s", ", ".join(unexpected))
        return missing, unexpected


def _not_applicable(name, why):
    class _NA(Algorithm):
        def __init__(self, *a, **k):
            raise NotImplementedError(f"{name}: {why}")
    _NA.__name__ = name
    return _NA


BlurPool = _not_applicable("BlurPool", "anti-aliased convolutions are a ResNet surgery; SwinV2 has none")
ChannelsLast = _not_applicable("ChannelsLast", "SwinV2 activations are token-major already")
ProgressiveResizing = _not_applicable("ProgressiveResizing",
                                      "SwinV2 has a fixed input resolution (PatchEmbed asserts it)")
