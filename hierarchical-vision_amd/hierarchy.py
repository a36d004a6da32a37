"""Taxonomy handling and hierarchical losses -- drop-in for hierarchy.py.

Host-side integer work (label parsing, tier-id assignment, parent lookup, the
leaf permutation that makes every taxonomy node a contiguous leaf range) is
plain Python/numpy and bit-exact with the reference.  The losses run as HIP
kernels (ops.multitask_cross_entropy, ops.hierarchical_cross_entropy).
"""
import collections
import dataclasses
import math
import os
import pathlib

import numpy as np
import torch

from . import ops

N_TIERS = 7


# --------------------------------------------------------------------------- labels
@dataclasses.dataclass(frozen=True)
class HierarchicalLabel:
    """`NNNNN_kingdom_phylum_class_order_family_genus_species` with every tier
    prefixed by its ancestors so repeated names on different branches stay
    distinct (hierarchy.py:230-330)."""
    raw: str
    number: int
    kingdom: str
    phylum: str
    cls: str
    order: str
    family: str
    genus: str
    species: str

    @classmethod
    def parse(cls, name):
        index, top, *tiers = name.split("_")
        cleaned, complete = [top], top
        for tier in tiers:
            complete = f"{complete}-{tier}"
            cleaned.append(complete)
        assert len(cleaned) == N_TIERS, f"{len(cleaned)} != {N_TIERS}"
        return cls(name, int(index), *cleaned)

    @property
    def clean_tiers(self):
        return [self.kingdom, self.phylum, self.cls, self.order, self.family, self.genus,
                self.species]

    @property
    def cleaned(self):
        return "_".join([str(self.number).rjust(5, "0")] + self.clean_tiers)

    def dist(self, other: "HierarchicalLabel") -> int:
        mine, theirs = self.clean_tiers, other.clean_tiers
        for level, t in enumerate(range(N_TIERS - 1, -1, -1)):
            if mine[t] == theirs[t]:
                return level
        return N_TIERS


def assign_tier_ids(class_names):
    """Tier ids in first-seen order over sorted() names (hierarchy.py:202-227).

    Returns (classes, {class: LongTensor[7]}, num_classes tuple)."""
    classes = sorted(class_names)
    lookup = [dict() for _ in range(N_TIERS)]
    out = {}
    for c in classes:
        ids = []
        for t, v in enumerate(HierarchicalLabel.parse(c).clean_tiers):
            ids.append(lookup[t].setdefault(v, len(lookup[t])))
        out[c] = torch.tensor(ids)
    return classes, out, tuple(len(d) for d in lookup)


class HierarchicalImageFolder:
    """Only the class-indexing half of the reference's image folder
    (hierarchy.py:188-227); image decoding is outside this hot path."""

    num_classes = None

    def find_classes(self, directory):
        names = [e.name for e in os.scandir(directory) if e.is_dir()]
        classes, class_to_idxs, self.num_classes = assign_tier_ids(names)
        return classes, class_to_idxs


def _split_class_names(directory):
    directory = pathlib.Path(directory)
    train = {p.stem for p in (directory / "train").iterdir()}
    val = {p.stem for p in (directory / "val").iterdir()}
    return sorted(train | val)


def build_parent_label_lookup(directory):
    """(n_tiers - 1) uint16 vectors child id -> parent id (hierarchy.py:429-485)."""
    return parent_vectors([HierarchicalLabel.parse(n) for n in _split_class_names(directory)])


def parent_vectors(labels):
    lookups = [dict() for _ in range(N_TIERS)]
    for label in labels:
        for i, v in enumerate(label.clean_tiers):
            lookups[i].setdefault(v, len(lookups[i]))
    vecs = []
    for i in range(1, N_TIERS):
        vec = np.zeros((len(lookups[i]),), dtype=np.uint16)
        for label in labels:
            t = label.clean_tiers
            vec[lookups[i][t[i]]] = lookups[i - 1][t[i - 1]]
        vecs.append(vec)
    return vecs


def build_tree_dist_matrix(labels):
    """uint8 [n, n] tree distances (hierarchy.py:391-426) from parsed labels,
    vectorised over the 7 tier-id columns."""
    _, c2i, _ = assign_tier_ids([lb.raw for lb in labels])
    ids = np.stack([c2i[lb.raw].numpy() for lb in sorted(labels, key=lambda x: x.raw)])
    dist = np.full((len(ids), len(ids)), N_TIERS, dtype=np.uint8)
    for lvl, t in enumerate(range(N_TIERS - 1, -1, -1)):
        same = ids[:, None, t] == ids[None, :, t]
        dist = np.where(same & (dist == N_TIERS), np.uint8(lvl), dist)
    return torch.from_numpy(dist)


# --------------------------------------------------------------------------- taxonomy
class Taxonomy:
    """Leaf paths of a 7-tier taxonomy plus the segment tables the HXE kernel scans.

    leaf_paths[k] = tier ids of leaf k (leaf id = species tier id = index of
    the class in sorted() order).  ``perm`` orders leaves lexicographically by
    their path, which makes every node's leaves one contiguous range
    [node_start, node_end) of permuted positions -- for iNat21-style names
    (numbered in taxonomic order) perm is the identity."""

    def __init__(self, class_names):
        self.classes, c2i, self.num_classes = assign_tier_ids(class_names)
        self.leaf_paths = np.stack([c2i[c].numpy() for c in self.classes]).astype(np.int64)
        if self.num_classes[-1] != len(self.classes):
            raise ValueError("every class must be its own leaf (distinct species paths)")
        self.perm = np.lexsort(self.leaf_paths.T[::-1]).astype(np.int32)
        self.identity_perm = bool(np.all(self.perm == np.arange(len(self.perm))))
        ordered = self.leaf_paths[self.perm]
        starts, ends = [], []
        for t in range(N_TIERS):
            n = self.num_classes[t]
            col = ordered[:, t]
            st = np.full(n, -1, np.int64)
            en = np.full(n, -1, np.int64)
            change = np.flatnonzero(np.r_[True, col[1:] != col[:-1]])
            bounds = np.r_[change, len(col)]
            for a, b in zip(bounds[:-1], bounds[1:]):
                node = col[a]
                if st[node] != -1:
                    raise ValueError(f"tier {t} node {node} is not contiguous in path order")
                st[node], en[node] = a, b
            starts.append(st)
            ends.append(en)
        self.node_start = np.concatenate(starts).astype(np.int32)
        self.node_end = np.concatenate(ends).astype(np.int32)
        self.tier_base = np.r_[0, np.cumsum(self.num_classes)[:-1]].astype(np.int32)
        self._dev = {}

    @property
    def num_leaves(self):
        return len(self.classes)

    @classmethod
    def from_directory(cls, directory):
        return cls(_split_class_names(directory))

    @classmethod
    def synthetic(cls, sizes=(3, 13, 51, 273, 1103, 4884, 10000)):
        """iNat21-shaped synthetic tree: parent of node i at
        tier t is floor(i * n_{t-1} / n_t)."""
        n_leaves = sizes[-1]
        names = []
        for leaf in range(n_leaves):
            ids = [0] * N_TIERS
            ids[-1] = leaf
            for t in range(N_TIERS - 2, -1, -1):
                ids[t] = ids[t + 1] * sizes[t] // sizes[t + 1]
            names.append("_".join([f"{leaf:05d}"] + [f"t{t}n{ids[t]}" for t in range(N_TIERS)]))
        return cls(names)

    def device_tables(self, device):
        """(perm or None, node_start, node_end, tier_base, leaf_paths) on `device`."""
        key = str(device)
        if key not in self._dev:
            mk = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
            self._dev[key] = (None if self.identity_perm else mk(self.perm), mk(self.node_start),
                              mk(self.node_end), mk(self.tier_base), mk(self.leaf_paths))
        return self._dev[key]


def hxe_level_coeffs(tree_weights="uniform", alpha=0.1):
    """Coefficients c_l of L = sum_l c_l LSE_l for levels l = 0 (leaf) .. 7 (root):
    L = -sum_{l<7} lambda_l (LSE_l - LSE_{l+1}), lambda_l = 1 (uniform) or
    exp(-alpha * l) (exponential; Bertinetto et al. 2020)."""
    if tree_weights == "uniform":
        lam = [1.0] * N_TIERS
    elif tree_weights == "exponential":
        lam = [math.exp(-alpha * l) for l in range(N_TIERS)]
    else:
        raise ValueError(tree_weights)
    c = [-lam[0]] + [lam[l - 1] - lam[l] for l in range(1, N_TIERS)] + [lam[-1]]
    return torch.tensor(c, dtype=torch.float32)


# --------------------------------------------------------------------------- heads
class MultitaskHead(torch.nn.Module):
    """One Linear per taxonomy tier on shared features (hierarchy.py:19-47)."""

    def __init__(self, num_features, num_classes):
        super().__init__()
        self.num_classes = tuple(num_classes)
        for n in self.num_classes:
            assert n > 0
        self.heads = torch.nn.ModuleList([torch.nn.Linear(num_features, n) for n in self.num_classes])

    def forward(self, x):
        from .options import OPTIONS
        ws = [h.weight for h in self.heads]
        if OPTIONS.head_gemm and torch.is_autocast_enabled() and ops.head_supported(x, ws):
            # all tiers as one GEMM over the concatenated classes (libhvk head kernels)
            return list(ops.head_linear(x, ws, [h.bias for h in self.heads]))
        return [head(x) for head in self.heads]


def multitask_surgery(model, head: str, num_classes):
    """Replace `model.<head>` with a MultitaskHead (hierarchy.py:50-62)."""
    if not hasattr(model, head):
        raise RuntimeError(f"model has no attribute {head}!")
    num_features = max(getattr(model, head).weight.shape)
    setattr(model, head, MultitaskHead(num_features, num_classes))


# --------------------------------------------------------------------------- losses
class MultitaskCrossEntropy(torch.nn.Module):
    """sum_l coeffs[l] * CE(inputs[l], targets[l]) (hierarchy.py:65-94), all tiers in
    one kernel launch.  targets: LongTensor [B, tiers], or a list of per-tier
    probability targets (LabelSmoothing)."""

    def __init__(self, *args, coeffs=(1.0,), **kwargs):
        super().__init__()
        if isinstance(coeffs, torch.Tensor):
            coeffs = coeffs.clone().detach().float()
        else:
            coeffs = torch.tensor(list(coeffs), dtype=torch.float)
        self.register_buffer("coeffs", coeffs)
        self._off = {}

    def _offsets(self, sizes, device):
        key = (tuple(sizes), str(device))
        if key not in self._off:
            self._off[key] = torch.tensor(np.r_[0, np.cumsum(sizes)], dtype=torch.int32, device=device)
        return self._off[key]

    def forward(self, inputs, targets):
        assert len(inputs) == len(self.coeffs), f"{len(inputs)} != {len(self.coeffs)}"
        sizes = [z.shape[1] for z in inputs]
        logits = torch.cat([z.float() for z in inputs], dim=1)
        off = self._offsets(sizes, logits.device)
        if isinstance(targets, list):
            assert len(targets) == len(inputs), f"{len(targets)} != {len(inputs)}"
            soft = torch.cat([t.float() for t in targets], dim=1)
            return ops.multitask_cross_entropy(logits, off, self.coeffs, soft=soft)
        assert targets.shape[1] == len(inputs)
        return ops.multitask_cross_entropy(logits, off, self.coeffs, targets=targets)


def soft_cross_entropy(input, target):
    """Flat CE for int or probability targets (composer.loss.soft_cross_entropy as
    called at models.py:112) -- one-head case of the multitask kernel."""
    off = torch.tensor([0, input.shape[1]], dtype=torch.int32, device=input.device)
    one = torch.ones(1, device=input.device)
    if target.dtype.is_floating_point:
        return ops.multitask_cross_entropy(input.float(), off, one, soft=target)
    return ops.multitask_cross_entropy(input.float(), off, one, targets=target.reshape(-1, 1))


class HierarchicalCrossEntropy(torch.nn.Module):
    """HXE (Bertinetto et al., CVPR 2020) over leaf logits.  The reference only
    stubs it (hierarchy.py:183-185) and exposes the knobs hxe_tree_weights /
    hxe_alpha (configs.py:93-96): parity unpinned, pinned by closed-form tests.

    forward(logits [B, n_leaves], targets [B, 7] tier ids or [B] leaf ids)."""

    def __init__(self, taxonomy: Taxonomy, tree_weights="uniform", alpha=0.1):
        super().__init__()
        self.taxonomy = taxonomy
        self.register_buffer("level_coeff", hxe_level_coeffs(tree_weights, alpha))

    def forward(self, logits, targets):
        if isinstance(targets, list) or targets.dtype.is_floating_point:
            raise NotImplementedError("HXE takes hard taxonomy targets (no label smoothing)")
        perm, start, end, base, paths = self.taxonomy.device_tables(logits.device)
        if targets.ndim == 1:
            targets = paths[targets]
        return ops.hierarchical_cross_entropy(logits, targets, perm, start, end, base,
                                              self.level_coeff)


# --------------------------------------------------------------------------- metrics
def fine_grained_predictions(output, topk=1, hierarchy_level=-1):
    """Top-k predictions of the finest tier (hierarchy.py:371-388)."""
    if isinstance(output, list):
        output = output[hierarchy_level]
    maxk = min(topk, output.shape[1])
    return output.topk(maxk, dim=1, largest=True, sorted=True)[1]


class _SumMetric(torch.nn.Module):
    """Minimal torchmetrics-style accumulator (update / compute / reset)."""

    def __init__(self):
        super().__init__()
        self.register_buffer("num", torch.zeros((), dtype=torch.float64))
        self.register_buffer("den", torch.zeros((), dtype=torch.float64))

    def reset(self):
        self.num.zero_()
        self.den.zero_()

    def compute(self):
        return (self.num / self.den).float()


class FineGrainedAccuracy(_SumMetric):
    """Top-k accuracy of the finest tier (hierarchy.py:97-123)."""

    def __init__(self, topk=1):
        super().__init__()
        self.topk = topk

    def update(self, outputs, targets):
        assert isinstance(outputs, list) and targets.ndim > 1
        preds = fine_grained_predictions(outputs, topk=self.topk).view(-1, self.topk)
        tgt = targets[:, -1].view(-1, 1).expand(preds.shape)
        self.num += (preds == tgt).sum()
        self.den += tgt.numel() / self.topk


class Accuracy(_SumMetric):
    """torchmetrics.Accuracy(task="multiclass", num_classes, top_k) with its default micro
    average, as models.py:87-97 builds it: a sample counts when its target is among the top_k
    logits.  Hard taxonomy targets [B, tiers] (the HXE variant's) score the leaf column."""

    def __init__(self, num_classes, top_k=1):
        super().__init__()
        if top_k > num_classes:
            raise ValueError(f"top_k ({top_k}) > num_classes ({num_classes})")
        self.num_classes = num_classes
        self.top_k = top_k

    def update(self, preds, targets):
        if targets.dtype.is_floating_point:
            raise ValueError("Accuracy takes integer class targets")
        if targets.ndim == 2:
            targets = targets[:, -1]
        top = preds.topk(self.top_k, dim=1, largest=True, sorted=True)[1]
        self.num += (top == targets.view(-1, 1)).any(dim=1).sum()
        self.den += targets.numel()


class TreeDistance(_SumMetric):
    """Mean tree distance of the top-1 prediction (hierarchy.py:126-154)."""

    def __init__(self, tree_dists):
        super().__init__()
        self.register_buffer("tree_dists", tree_dists)

    def update(self, outputs, targets):
        preds = fine_grained_predictions(outputs, topk=1).squeeze()
        targets = targets.squeeze()
        self.num += self.tree_dists[preds, targets].sum()
        self.den += targets.numel()


class FineGrainedTreeDistance(TreeDistance):
    def update(self, outputs, targets):
        assert isinstance(outputs, list) and targets.ndim > 1
        super().update(outputs[-1], targets[:, -1])


class CrossEntropyMetric(_SumMetric):
    """Running mean cross-entropy (composer.metrics.CrossEntropy semantics)."""

    def update(self, preds, targets):
        if not targets.dtype.is_floating_point and targets.ndim == 2:
            targets = targets[:, -1]  # HXE: [B, tiers] taxonomy targets, the leaf column
        b = preds.shape[0]
        self.num += soft_cross_entropy(preds, targets).detach().double() * b
        self.den += b


class FineGrainedCrossEntropy(CrossEntropyMetric):
    """CE of the finest tier only (hierarchy.py:170-180)."""

    def update(self, preds, targets):
        if not isinstance(preds, list):
            raise RuntimeError("FineGrainedCrossEntropy needs a list of predictions")
        super().update(preds[-1], targets[:, -1])


class LeafCountLookup:
    """Leaves under every node, for split tooling (hierarchy.py:333-368)."""

    def __init__(self, labels):
        self._lookup = collections.defaultdict(int)
        for label in labels:
            for name, v in zip(("kingdom", "phylum", "cls", "order", "family", "genus", "species"),
                               label.clean_tiers):
                self._lookup[(v, name)] += 1
        self.total = len(labels)

    def closest(self, n):
        if isinstance(n, float):
            assert 0 <= n <= 1, "n must be fractional"
            n = int(self.total * n)
        best, dist = None, float("inf")
        for label, count in self._lookup.items():
            if abs(count - n) < dist:
                best, dist = (*label, count), abs(count - n)
        if best is None:
            raise RuntimeError("no values in lookup!")
        return best
