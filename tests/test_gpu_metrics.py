"""On-device eval metrics (hierarchy.py:97-180) and the uint8 tree-distance matrix
(hierarchy.py:391-426) on the GPU against plain-Python restatements / the reference's own
distances (taxonomy_golden hand.dist)."""
import numpy as np
import pytest
import torch

from oracle import hierarchy_ref

pytestmark = pytest.mark.gpu


def _outputs(B, sizes, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return [torch.randn(B, n, device="cuda", generator=g) for n in sizes]


@pytest.mark.parametrize("topk", [1, 5])
def test_fine_grained_accuracy(topk):
    from hvamd.hierarchy import FineGrainedAccuracy
    sizes = (3, 4, 5, 6, 7, 8, 40)
    m = FineGrainedAccuracy(topk=topk).cuda()
    hits = tot = 0
    for step in range(3):
        outs = _outputs(64, sizes, step)
        tgt = torch.stack([torch.randint(0, n, (64,), device="cuda") for n in sizes], 1)
        tgt[::3, -1] = outs[-1][::3].argmax(1)  # some hits for sure
        m.update(outs, tgt)
        z, t = outs[-1].cpu().numpy(), tgt[:, -1].cpu().numpy()
        for b in range(64):
            top = np.argsort(-z[b], kind="stable")[:topk]
            hits += int(t[b] in top)
        tot += 64
    assert abs(m.compute().item() - hits / tot) < 1e-6


def test_tree_distance_matches_reference_distances(golden):
    """build_tree_dist_matrix (uint8, vectorised over tier ids) == the reference's pairwise
    HierarchicalLabel.dist on the hand-made classes; FineGrainedTreeDistance averages the
    distance of each top-1 prediction to its target on the device."""
    from hvamd.hierarchy import FineGrainedTreeDistance, HierarchicalLabel, build_tree_dist_matrix
    g = golden("taxonomy_golden")
    labels = [HierarchicalLabel.parse(c) for c in g["hand.classes"]]
    mat = build_tree_dist_matrix(labels)
    assert mat.dtype == torch.uint8 and np.array_equal(mat.numpy(), g["hand.dist"])
    names = hierarchy_ref.synthetic_inat_names((2, 3, 4, 5, 6, 7, 30))
    labels = [HierarchicalLabel.parse(n) for n in names]
    mat = build_tree_dist_matrix(labels)
    ref = np.array([[hierarchy_ref.tree_dist(a, b) for b in sorted(names)] for a in sorted(names)])
    assert np.array_equal(mat.numpy(), ref)
    m = FineGrainedTreeDistance(mat.cuda()).cuda()
    outs = _outputs(50, (2, 3, 4, 5, 6, 7, 30), 3)
    tgt = torch.randint(0, 30, (50, 7), device="cuda")
    m.update(outs, tgt)
    pred = outs[-1].argmax(1).cpu().numpy()
    want = np.mean([ref[p, t] for p, t in zip(pred, tgt[:, -1].cpu().numpy())])
    assert abs(m.compute().item() - want) < 1e-6


def test_fine_grained_cross_entropy():
    from hvamd.hierarchy import FineGrainedCrossEntropy
    m = FineGrainedCrossEntropy().cuda()
    outs = _outputs(32, (3, 5, 100), 4)
    tgt = torch.stack([torch.randint(0, n, (32,), device="cuda") for n in (3, 5, 100)], 1)
    m.update(outs, tgt)
    want = torch.nn.functional.cross_entropy(outs[-1].cpu(), tgt[:, -1].cpu()).item()
    assert abs(m.compute().item() - want) < 1e-5 * abs(want)
    with pytest.raises(RuntimeError):
        m.update(outs[-1], tgt)
