"""Two ranks on the real product path: SwinV2 (libhvk kernels) + HXE + the Trainer's bucketed
hook-driven all-reduce + the fused DecoupledSGDW step (1/world mean, clipping and EMA folded in),
with half the batch per rank, must match one process stepping on the whole batch (main.py:44-48
batch split, :104-124 DDP).  Both ranks share the box's one GPU, so the exchange runs over gloo
(CUDA tensors staged through the host); RCCL over xGMI runs the same hooks in bench.py."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
TAX_SIZES = (2, 3, 4, 5, 6, 7, 12)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(rank, world, port, out, steps=2):
    from hvamd import hierarchy, models, optim, swinv2
    from hvamd.algorithmic import EMA, GradientClipping
    from hvamd.trainer import Trainer
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    tax = hierarchy.Taxonomy.synthetic(TAX_SIZES)
    net = swinv2.SwinTransformerV2(img_size=56, embed_dim=32, depths=[2, 2], num_heads=[1, 2],
                                   window_size=7, num_classes=tax.num_leaves,
                                   drop_path_rate=0.0).to(dev)
    loss_fn = hierarchy.HierarchicalCrossEntropy(tax, tree_weights="exponential").to(dev)
    model = models.Model(net, None, None, loss_fn)
    opt = optim.DecoupledSGDW(optim.set_weight_decay(model), lr=0.05, momentum=0.9,
                              weight_decay=5e-4)
    ema = EMA(half_life="4ba", update_interval="1ba")
    trainer = Trainer(model, opt, [GradientClipping("norm", 1e4), ema], bucket_mb=0.05)
    if world > 1:
        assert len(trainer.buckets.buckets) > 2
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(4, 3, 56, 56, device=dev, generator=g)
    y = torch.tensor(tax.leaf_paths[[1, 5, 9, 11]], device=dev)
    per = 4 // world
    sl = slice(rank * per, rank * per + per)
    p0 = [p.detach().clone() for p in model.parameters()]
    for _ in range(steps):
        trainer.train_step((x[sl], y[sl]))
    torch.cuda.synchronize()
    # one more step under the profiler: the elementwise adds it launches (gradient sums)
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        trainer.train_step((x[sl], y[sl]))
        torch.cuda.synchronize()
    adds = sum(1 for e in prof.events() if "CUDAFunctor_add" in e.name)
    # what the steps moved: the update (and the EMA's pull) itself, not the weights around it
    out[rank] = ([(p.detach() - q).cpu().numpy() for p, q in zip(model.parameters(), p0)],
                 [(e - q).cpu().numpy() for e, q in zip(ema.ema_params, p0)], opt._fused is not None,
                 adds)
    if world > 1:
        dist.destroy_process_group()


def test_two_ranks_equal_one_process_full_batch():
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_run, args=(2, _free_port(), out), nprocs=2, join=True)
    single = {}
    _run(0, 1, 0, single)
    assert out[0][2] and single[0][2]  # the fused optimizer step ran on both sides
    # the bucketed exchange adds no gradient pass: autograd hands each weight gradient over
    # (.grad is None between steps) and the hook copies it into the bucket -- the elementwise
    # adds of a world-2 step are the model's own (e.g. proj.weight's two contributions)
    assert out[0][3] == single[0][3] and out[1][3] == single[0][3], (out[0][3], out[1][3], single[0][3])
    # parameter and EMA deltas over the two steps; per-rank weight-gradient reductions run over
    # half the tokens (another chunking) and the backward's bias-table atomics sum in a
    # run-dependent order: 2e-2 per tensor bounds it (a missing 1/world would be 100 %)
    for r in range(2):
        for a, b in zip(out[r][0] + out[r][1], single[0][0] + single[0][1]):
            a, b = torch.from_numpy(a), torch.from_numpy(b)
            rel = ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
            assert rel < 2e-2, (r, rel)


def test_rccl_one_rank_buckets_match_plain_step():
    """The RCCL (nccl backend) path on hardware: a one-rank process group with the buckets
    forced on runs the hook-launched all-reduces on RCCL's stream, synchronize() and the
    fused step on the bucket views; with one rank the exchange is the identity, so two steps
    must equal two steps without buckets up to the run-to-run order of the backward's
    bias-table atomics (1e-3 relative per tensor: measured up to 1.9e-4 between runs; a lost,
    doubled or stale gradient is O(1))."""
    from hvamd import hierarchy, models, optim, swinv2
    from hvamd.algorithmic import GradientClipping
    from hvamd.ddp import GradientBuckets
    from hvamd.trainer import Trainer
    dev = torch.device("cuda:0")

    def run(bucketed):
        torch.manual_seed(0)
        tax = hierarchy.Taxonomy.synthetic(TAX_SIZES)
        net = swinv2.SwinTransformerV2(img_size=56, embed_dim=32, depths=[2, 2], num_heads=[1, 2],
                                       window_size=7, num_classes=tax.num_leaves,
                                       drop_path_rate=0.0).to(dev)
        loss_fn = hierarchy.HierarchicalCrossEntropy(tax, tree_weights="exponential").to(dev)
        model = models.Model(net, None, None, loss_fn)
        opt = optim.DecoupledSGDW(optim.set_weight_decay(model), lr=0.05, momentum=0.9,
                                  weight_decay=5e-4)
        trainer = Trainer(model, opt, [GradientClipping("norm", 1e4)])
        if bucketed:
            trainer.buckets = GradientBuckets(model, bucket_mb=0.05, force=True)
            assert trainer.buckets.enabled and len(trainer.buckets.buckets) > 2
        g = torch.Generator(device=dev).manual_seed(1)
        x = torch.randn(4, 3, 56, 56, device=dev, generator=g)
        y = torch.tensor(tax.leaf_paths[[1, 5, 9, 11]], device=dev)
        for _ in range(2):
            trainer.train_step((x, y))
        torch.cuda.synchronize()
        return [p.detach().cpu().clone() for p in model.parameters()]

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        a = run(True)
    finally:
        dist.destroy_process_group()
    b = run(False)
    for u, v in zip(a, b):
        rel = ((u - v).norm() / v.norm().clamp_min(1e-12)).item()
        assert rel < 1e-3, rel
