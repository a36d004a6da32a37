"""Graph-mode training (Trainer.capture / replay: the step as two HIP graphs) gives the same
parameters as eager steps from the same start (drop-path off: no RNG in the step)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(seed=0):
    from hvamd import hierarchy, models, optim, swinv2
    from hvamd.algorithmic import GradientClipping
    from hvamd.trainer import Trainer
    torch.manual_seed(seed)
    dev = torch.device("cuda:0")
    tax = hierarchy.Taxonomy.synthetic((2, 3, 4, 5, 6, 7, 12))
    net = swinv2.SwinTransformerV2(img_size=56, embed_dim=32, depths=[2, 2], num_heads=[1, 2],
                                   window_size=7, num_classes=tax.num_leaves,
                                   drop_path_rate=0.0).to(dev)
    loss_fn = hierarchy.HierarchicalCrossEntropy(tax, tree_weights="exponential").to(dev)
    model = models.Model(net, None, None, loss_fn)
    return tax, model, dev


def _trainer(model):
    from hvamd import optim
    from hvamd.algorithmic import GradientClipping
    from hvamd.trainer import Trainer
    opt = optim.DecoupledSGDW(optim.set_weight_decay(model), lr=0.05, momentum=0.9,
                              weight_decay=5e-4)
    return Trainer(model, opt, [GradientClipping("norm", 2.0)])


def test_graph_replay_matches_eager():
    tax, model, dev = _setup()
    model_b = copy.deepcopy(model)
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(4, 3, 56, 56, device=dev, generator=g)
    y = torch.tensor(tax.leaf_paths[[1, 5, 9, 11]], device=dev)
    ta, tb = _trainer(model), _trainer(model_b)
    la = [ta.train_step((x, y)) for _ in range(6)]
    tb.capture((x, y), warmup=3)      # 3 eager steps inside, then capture
    lb = [tb.replay().clone() for _ in range(3)]
    torch.cuda.synchronize()
    for a, b in zip(la[3:], lb):
        assert abs(a.item() - b.item()) < 1e-3 * max(1.0, abs(a.item())), (a.item(), b.item())
    # the backward's f32 atomics (bias-table / bias gradients) sum in a run-dependent order, and
    # 6 SGD steps amplify that rounding noise in the smallest tensors: 1e-2 bounds it
    for (na, pa), (nb, pb) in zip(model.named_parameters(), model_b.named_parameters()):
        rel = ((pa - pb).norm() / pa.norm().clamp_min(1e-12)).item()
        assert rel < 1e-2, (na, rel)


def test_graph_replay_follows_lr_schedule():
    """A learning-rate change between replays reaches the captured fused update (lr / decay
    read from a device array refreshed before each replay) exactly as it reaches eager steps."""
    tax, model, dev = _setup()
    model_b = copy.deepcopy(model)
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(4, 3, 56, 56, device=dev, generator=g)
    y = torch.tensor(tax.leaf_paths[[1, 5, 9, 11]], device=dev)
    ta, tb = _trainer(model), _trainer(model_b)
    for _ in range(4):
        ta.train_step((x, y))
    tb.capture((x, y), warmup=3)
    tb.replay()
    for lr in (0.2, 0.0):  # a larger step, then none: the weights must not move on lr 0
        for t in (ta, tb):
            for grp in t.optimizer.param_groups:
                grp["lr"] = lr
        ta.train_step((x, y))
        tb.replay()
        if lr == 0.0:
            before = [p.detach().clone() for p in model_b.parameters()]
            tb.replay()
            torch.cuda.synchronize()
            for b, p in zip(before, model_b.parameters()):
                assert torch.equal(b, p.detach())
            ta.train_step((x, y))
    torch.cuda.synchronize()
    for (na, pa), (nb, pb) in zip(model.named_parameters(), model_b.named_parameters()):
        rel = ((pa - pb).norm() / pa.norm().clamp_min(1e-12)).item()
        assert rel < 1e-2, (na, rel)


def test_eager_step_after_capture_takes_current_lr():
    """After capture() the fused update reads lr / decay from a device array only inside the
    captured graph: an eager step after an lr change (e.g. the warm-up steps of a second
    capture) must use the new lr, not the value of the last replay's refresh."""
    tax, model, dev = _setup()
    model_b = copy.deepcopy(model)
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(4, 3, 56, 56, device=dev, generator=g)
    y = torch.tensor(tax.leaf_paths[[1, 5, 9, 11]], device=dev)
    ta, tb = _trainer(model), _trainer(model_b)
    for _ in range(4):
        ta.train_step((x, y))
    tb.capture((x, y), warmup=3)
    tb.replay()
    torch.cuda.synchronize()
    for t in (ta, tb):
        for grp in t.optimizer.param_groups:
            grp["lr"] = 0.0  # an eager step at lr 0 moves only by weight decay (decay = 1 at lr 0)
    before = [p.detach().clone() for p in model_b.parameters()]
    tb.train_step((x, y))
    torch.cuda.synchronize()
    for (n, p), b in zip(model_b.named_parameters(), before):
        assert torch.equal(b, p.detach()), n


def test_eager_step_after_replay_matches_eager_trainer():
    """An eager train_step after capture()/replay() computes this step's gradient alone: the
    captured gradient tensors .grad still points at must not be accumulated onto.
    Parameters AND momentum buffers after one more eager step at a nonzero lr equal those of
    a trainer that only ever stepped eagerly."""
    tax, model, dev = _setup()
    model_b = copy.deepcopy(model)
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(4, 3, 56, 56, device=dev, generator=g)
    y = torch.tensor(tax.leaf_paths[[1, 5, 9, 11]], device=dev)
    ta, tb = _trainer(model), _trainer(model_b)
    for _ in range(5):
        ta.train_step((x, y))
    tb.capture((x, y), warmup=3)
    tb.replay()
    tb.train_step((x, y))
    torch.cuda.synchronize()
    pairs = list(zip(model.named_parameters(), model_b.named_parameters()))
    for (na, pa), (_, pb) in pairs:
        rel = ((pa - pb).norm() / pa.norm().clamp_min(1e-12)).item()
        assert rel < 1e-2, (na, rel)
        ma = ta.optimizer.state[pa]["momentum_buffer"]
        mb = tb.optimizer.state[pb]["momentum_buffer"]
        rel = ((ma - mb).norm() / ma.norm().clamp_min(1e-12)).item()
        assert rel < 5e-2, ("momentum", na, rel)
