"""ORACLE (test infrastructure only) -- taxonomy work of hierarchy.py.

Pure-Python / numpy restatement (float64 for the losses) used to check the
product's host-side taxonomy tables and the HIP loss kernels.
"""
import math

import numpy as np

N_TIERS = 7


def parse_tiers(name: str) -> list:
    """HierarchicalLabel.parse (hierarchy.py:242-286): 'NNNNN_k_p_c_o_f_g_s' ->
    7 prefix-joined tier strings ('k', 'k-p', 'k-p-c', ...)."""
    parts = name.split("_")
    int(parts[0])  # the reference requires a numeric index (hierarchy.py:275)
    tiers, acc = [], None
    for p in parts[1:]:
        acc = p if acc is None else acc + "-" + p
        tiers.append(acc)
    assert len(tiers) == N_TIERS, f"{len(tiers)} != {N_TIERS}"
    return tiers


def find_classes(class_names):
    """HierarchicalImageFolder.find_classes (hierarchy.py:202-227).

    Returns (classes, {class: [7 tier ids]}, num_classes).  Ids per tier are
    handed out in first-seen order while walking sorted() class names."""
    classes = sorted(class_names)
    lookup = [dict() for _ in range(N_TIERS)]
    out = {}
    for c in classes:
        ids = []
        for t, v in enumerate(parse_tiers(c)):
            if v not in lookup[t]:
                lookup[t][v] = len(lookup[t])
            ids.append(lookup[t][v])
        out[c] = ids
    return classes, out, tuple(len(d) for d in lookup)


def parent_lookup(class_names):
    """build_parent_label_lookup (hierarchy.py:429-485) minus the directory
    walk: 6 uint16 vectors, vec[t-1][id at tier t] = id at tier t-1."""
    classes = sorted(set(class_names))
    lookup = [dict() for _ in range(N_TIERS)]
    paths = [parse_tiers(c) for c in classes]
    for p in paths:
        for t, v in enumerate(p):
            lookup[t].setdefault(v, len(lookup[t]))
    vecs = []
    for t in range(1, N_TIERS):
        vec = np.zeros(len(lookup[t]), np.uint16)
        for p in paths:
            vec[lookup[t][p[t]]] = lookup[t - 1][p[t - 1]]
        vecs.append(vec)
    return vecs


def tree_dist(a: str, b: str) -> int:
    """HierarchicalLabel.dist (hierarchy.py:315-330) on raw names."""
    ta, tb = parse_tiers(a), parse_tiers(b)
    for lvl, t in enumerate(range(N_TIERS - 1, -1, -1)):
        if ta[t] == tb[t]:
            return lvl
    return N_TIERS


def _log_softmax(z):
    z = np.asarray(z, np.float64)
    m = z.max(axis=-1, keepdims=True)
    return z - m - np.log(np.exp(z - m).sum(axis=-1, keepdims=True))


def cross_entropy(logits, target):
    """torch.nn.CrossEntropyLoss(reduction='mean'): int targets [B] or
    probability targets [B, K] (sum over classes, mean over batch)."""
    lp = _log_softmax(logits)
    target = np.asarray(target)
    if target.ndim == 1:
        return float(-lp[np.arange(lp.shape[0]), target].mean())
    return float(-(target * lp).sum(axis=-1).mean())


def multitask_cross_entropy(inputs, targets, coeffs):
    """MultitaskCrossEntropy.forward (hierarchy.py:76-94): hard targets
    [B, tiers] or a list of per-tier soft targets."""
    if not isinstance(targets, list):
        targets = list(np.asarray(targets).T)
    assert len(inputs) == len(targets) == len(coeffs)
    return float(sum(c * cross_entropy(z, t) for c, z, t in zip(coeffs, inputs, targets)))


def smooth_labels(n_classes, target, smoothing):
    """algorithmic.smooth_labels (algorithmic.py:160-164)."""
    oh = np.eye(n_classes)[np.asarray(target)]
    return oh * (1.0 - smoothing) + smoothing / n_classes


def hxe_level_weights(tree_weights: str, alpha: float):
    """lambda_l for l = 0 (leaf term) .. 6 (top tier | root)."""
    if tree_weights == "uniform":
        return [1.0] * N_TIERS
    if tree_weights == "exponential":
        return [math.exp(-alpha * l) for l in range(N_TIERS)]
    raise ValueError(tree_weights)


def hxe_loss(logits, leaf_paths, targets, lambdas):
    """Hierarchical cross-entropy (Bertinetto et al., CVPR 2020).  NOT
    implemented by the reference (hierarchy.py:183-185) -> PARITY UNPINNED.

    logits [B, L] leaf logits; leaf_paths [L, 7] tier ids of every leaf;
    targets [B, 7] tier ids (or [B] leaf ids).  With C(l) the ancestor of the
    target at level l (l = 0 leaf ... 6 top tier, 7 = root),
        log p(C(l)) = LSE_{k in leaves(C(l))} z_k - LSE_all z
        L_b = -sum_l lambda_l [log p(C(l)) - log p(C(l+1))],  log p(root) = 0
    and the batch loss is the mean of L_b."""
    z = np.asarray(logits, np.float64)
    paths = np.asarray(leaf_paths)
    targets = np.asarray(targets)
    if targets.ndim == 1:
        targets = paths[targets]
    total = 0.0
    for b in range(z.shape[0]):
        lse_all = _lse(z[b])
        logp = []
        for l in range(N_TIERS):
            t = N_TIERS - 1 - l
            members = paths[:, t] == targets[b, t]
            logp.append(_lse(z[b][members]) - lse_all)
        logp.append(0.0)
        total += -sum(lambdas[l] * (logp[l] - logp[l + 1]) for l in range(N_TIERS))
    return total / z.shape[0]


def _lse(v):
    v = np.asarray(v, np.float64)
    m = v.max()
    return float(m + np.log(np.exp(v - m).sum()))


def synthetic_inat_names(sizes=(3, 13, 51, 273, 1103, 4884, 10000)):
    """Synthetic iNat21-shaped tree used by tests and bench (SURVEY.md
    §8(c)(6)): tier sizes 3/13/51/273/1103/4884/10000, parent(i) at tier t =
    floor(i * n_{t-1} / n_t), names '%05d_t0x_t1y_...'."""
    n_leaves = sizes[-1]
    names = []
    for leaf in range(n_leaves):
        ids = [0] * N_TIERS
        ids[-1] = leaf
        for t in range(N_TIERS - 2, -1, -1):
            ids[t] = ids[t + 1] * sizes[t] // sizes[t + 1]
        parts = [f"{leaf:05d}"] + [f"t{t}n{ids[t]}" for t in range(N_TIERS)]
        names.append("_".join(parts))
    return names


def hxe_loss_torch(logits, paths, perm, node_start, node_end, tier_base, lambdas):
    """torch (autograd-capable, CPU) form of hxe_loss for the CPU baseline and
    for gradient checks.  paths: [B, 7] tier ids; perm / node_* / tier_base as
    in hvamd.hierarchy.Taxonomy (numpy)."""
    import torch
    z = logits[:, torch.as_tensor(perm, dtype=torch.long)]
    total = logits.new_zeros(())
    for b in range(z.shape[0]):
        lse = []
        for l in range(N_TIERS):
            t = N_TIERS - 1 - l
            k = tier_base[t] + int(paths[b, t])
            lse.append(torch.logsumexp(z[b, node_start[k]:node_end[k]], dim=0))
        lse.append(torch.logsumexp(z[b], dim=0))
        total = total - sum(lambdas[l] * (lse[l] - lse[l + 1]) for l in range(N_TIERS))
    return total / z.shape[0]
