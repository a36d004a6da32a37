"""Structured run configuration -- the schema of the reference's configs.py with a
YAML layering loader that needs no OmegaConf (default <- machine <- exp files,
left to right, as main.py:139-147 merges them)."""
import dataclasses
from dataclasses import dataclass, field
from typing import Any, Optional

import yaml

Args = dict  # str -> Any


@dataclass
class ModelConfig:
    name: str = "resnet50"
    variant: str = "full-tuning"  # full-tuning | linear-probe | simpleshot[-l2n|-cl2n]
    pretrained_checkpoint: Optional[str] = None


@dataclass
class DatasetConfig:
    path: str = ""
    resize_size: int = -1
    crop_size: int = 224
    global_batch_size: int = 2048
    drop_last: bool = False
    shuffle: bool = False
    channel_mean: tuple = (0.463, 0.480, 0.376)
    channel_std: tuple = (0.238, 0.229, 0.247)


@dataclass
class MachineConfig:
    datasets: dict = field(default_factory=dict)
    save_root: str = "."


@dataclass
class OptimConfig:
    name: str = "DecoupledSGDW"
    lr: float = 2.048
    momentum: float = 0.875
    weight_decay: float = 5e-4


@dataclass
class SchedulerConfig:
    name: str = "CosineAnnealingWithWarmupScheduler"
    args: dict = field(default_factory=lambda: {"t_warmup": "8ep", "alpha_f": 0.0})


@dataclass
class SaveConfig:
    interval: Optional[str] = "10ep"
    num_checkpoints_to_keep: int = 1
    overwrite: bool = True
    wandb: bool = True


@dataclass
class WandbConfig:
    entity: str = "imageomics"
    project: str = "hierarchical-vision"


@dataclass
class SimpleShotConfig:
    centered: bool = False
    l2_normalized: bool = False
    hierarchical: bool = False


@dataclass
class AlgorithmConfig:
    cls: str = ""
    args: dict = field(default_factory=dict)


@dataclass
class HierarchyConfig:
    variant: str = ""  # "" | "multitask" | "hxe"
    multitask_coeffs: list = field(default_factory=list)
    hxe_tree_weights: str = "uniform"  # uniform | exponential
    hxe_alpha: float = 0.1


@dataclass
class Config:
    run_name: str = "base"
    is_train: bool = True
    seed: int = 42
    max_duration: str = "90ep"
    grad_accum: Any = "auto"
    load_path: Optional[str] = None
    tags: list = field(default_factory=list)
    hierarchy: HierarchyConfig = field(default_factory=HierarchyConfig)
    model: ModelConfig = field(default_factory=ModelConfig)
    train_dataset: DatasetConfig = field(default_factory=DatasetConfig)
    eval_dataset: DatasetConfig = field(default_factory=DatasetConfig)
    optim: OptimConfig = field(default_factory=OptimConfig)
    scheduler: SchedulerConfig = field(default_factory=SchedulerConfig)
    algorithms: list = field(default_factory=list)
    machine: MachineConfig = field(default_factory=MachineConfig)
    save: SaveConfig = field(default_factory=SaveConfig)
    wandb: WandbConfig = field(default_factory=WandbConfig)
    simpleshot: SimpleShotConfig = field(default_factory=SimpleShotConfig)


def _merge(obj, data, path="config"):
    if not isinstance(data, dict):
        raise TypeError(f"{path}: expected a mapping, got {type(data).__name__}")
    for key, val in data.items():
        if not hasattr(obj, key):
            raise KeyError(f"{path}.{key} is not a config field")
        cur = getattr(obj, key)
        if dataclasses.is_dataclass(cur):
            _merge(cur, val or {}, f"{path}.{key}")
        elif key == "algorithms":
            setattr(obj, key, [AlgorithmConfig(cls=a["cls"], args=dict(a.get("args") or {}))
                               for a in (val or [])])
        else:
            setattr(obj, key, val)


def merge(config: Config, *layers) -> Config:
    """Apply dict layers (e.g. parsed YAML files) onto `config`, left to right."""
    for layer in layers:
        _merge(config, layer or {})
    return config


def load_config(*files, overrides=None) -> Config:
    """Config() <- each YAML file in order <- overrides (dict)."""
    cfg = Config()
    for f in files:
        if not f:
            continue
        with open(f) as fd:
            merge(cfg, yaml.safe_load(fd))
    if overrides:
        merge(cfg, overrides)
    return cfg
