"""World-size-2 gloo run of the gradient exchange (hvamd.ddp.GradientBuckets) on CPU:
bucketed, hook-driven all-reduce must equal the full-batch gradient of one process."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _net():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.GELU(), torch.nn.Linear(32, 32),
                               torch.nn.LayerNorm(32), torch.nn.Linear(32, 4))


def _data():
    g = torch.Generator().manual_seed(1)
    return torch.randn(8, 16, generator=g), torch.randint(0, 4, (8,), generator=g)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hvamd.ddp import GradientBuckets
    net = _net()
    # tiny buckets so several all-reduces are in flight during backward
    buckets = GradientBuckets(net, bucket_mb=0.002)
    assert len(buckets.buckets) > 2
    x, y = _data()
    shard = slice(rank * 4, rank * 4 + 4)
    for step in range(2):
        loss = torch.nn.functional.cross_entropy(net(x[shard]), y[shard])
        loss.backward()
        buckets.synchronize()
        if step == 0:
            grads = [p.grad.clone() for p in net.parameters()]
        buckets.reset()
    out[rank] = [g.numpy() for g in grads]
    dist.destroy_process_group()


def test_bucketed_allreduce_equals_full_batch_gradient():
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    net = _net()
    x, y = _data()
    torch.nn.functional.cross_entropy(net(x), y).backward()
    for r in range(2):
        for g, p in zip(out[r], net.parameters()):
            assert torch.allclose(torch.from_numpy(g), p.grad, atol=1e-6), r


def _worker_views(rank, world, port, out):
    """After the exchange every grad is a view into its bucket (the optimizer's flat
    buffers), a parameter that got no gradient reads zeros, the first bucket is the small
    one, and between steps .grad is None (autograd hands the new gradient over: no
    grad += new, no zero pass)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hvamd.ddp import GradientBuckets
    net = _net()
    net.unused = torch.nn.Parameter(torch.ones(5))
    buckets = GradientBuckets(net, bucket_mb=0.004, first_mb=0.0005, last_mb=0.0025)
    sizes = [b[0].numel() for b in buckets.buckets]
    head_w = net[4].weight  # the last layer's weight: ready first in the backward
    bucket_of = {id(p): i for i, (_, ps) in enumerate(buckets.buckets) for p in ps}
    res = {"first_small": sizes[0] <= 0.0005 * 2 ** 18 + 32 * 32 and sizes[0] < max(sizes),
           # the head weight rides in the FIRST bucket (it once waited in bucket 1 behind a
           # 40 KB head-bias bucket), the first-registered Linear in the small LAST one
           "head_weight_first_bucket": bucket_of[id(head_w)] == 0,
           "embed_last_bucket": bucket_of[id(net[0].weight)] == len(sizes) - 1 and sizes[-1] <= 0.0025 * 2 ** 18}
    x, y = _data()
    res["none_before"] = all(p.grad is None for p in net.parameters())
    ok_views, unused_zero = True, True
    for step in range(2):
        torch.nn.functional.cross_entropy(net(x[rank * 4:rank * 4 + 4]), y[rank * 4:rank * 4 + 4]).backward()
        buckets.synchronize()
        flats = buckets.flat_buffers()
        for p in net.parameters():
            base = p.grad.data_ptr()
            ok_views &= any(f.data_ptr() <= base < f.data_ptr() + 4 * f.numel() for f in flats)
        unused_zero &= bool((net.unused.grad == 0).all())
        buckets.reset()
        res["none_after_reset"] = all(p.grad is None for p in net.parameters())
    res["views"] = ok_views
    res["unused_zero"] = unused_zero
    out[rank] = res
    dist.destroy_process_group()


def test_bucket_plan_swinv2t_hxe_sizes():
    """The bucket plan on SwinV2-T + a 10 000-leaf HXE head's real parameter sizes (built on
    the CPU): the head weight (30.7 MB, larger than first_mb) forms the first bucket
    with the head bias, every middle bucket stays <= 64 MB, and the last bucket -- the exposed
    tail after the backward -- holds <= 4 MB of the earliest layers."""
    from hvamd.ddp import GradientBuckets
    from hvamd.swinv2 import SwinTransformerV2
    m = SwinTransformerV2(num_classes=10000)
    names = [n for n, p in m.named_parameters() if p.requires_grad]
    numels = [p.numel() for p in m.parameters() if p.requires_grad]
    plan = GradientBuckets.plan(numels)
    mb = [4 * sum(numels[i] for i in b) / 2 ** 20 for b in plan]
    assert sorted(i for b in plan for i in b) == list(range(len(numels)))
    assert names.index("head.weight") in plan[0] and names.index("head.bias") in plan[0]
    assert 8 <= mb[0] <= 40
    assert all(x <= 64 for x in mb[1:-1])
    assert mb[-1] <= 4 and names.index("patch_embed.proj.weight") in plan[-1]
    assert len(plan) >= 4


def test_bucket_views_unused_params_small_first_bucket():
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker_views, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        assert all(out[r].values()), out[r]


# ---------------------------------------------------------------- the real Trainer, world 2
MINI = dict(img_size=56, embed_dim=32, depths=(2, 2), num_heads=(1, 2), window_size=7)
TAX_SIZES = (2, 3, 4, 5, 6, 7, 12)


class _OracleSwin(torch.nn.Module):
    """CPU stand-in for the SwinV2 module (whose ops are GPU-only): the oracle's f32
    restatement (swinv2.py semantics) with its parameters as nn.Parameters, behind the
    ComposerModel surface the Trainer drives (forward(batch), loss(outputs, batch))."""

    def __init__(self, tax):
        super().__init__()
        from oracle import hierarchy_ref, swinv2_ref
        self.ref, self.href = swinv2_ref, hierarchy_ref
        shapes = swinv2_ref.state_shapes(num_classes=tax.num_leaves, **MINI)
        init = swinv2_ref.init_params_from_rng(shapes, 3)
        self.names = sorted(init)
        self.ps = torch.nn.ParameterList([torch.nn.Parameter(init[n]) for n in self.names])
        self.geom = swinv2_ref.model_geometry(**MINI)
        self.tax = tax
        self.lam = hierarchy_ref.hxe_level_weights("exponential", 0.1)

    def forward(self, batch):
        return self.ref.forward(dict(zip(self.names, self.ps)), batch[0], self.geom)

    def loss(self, outputs, batch):
        t = self.tax
        return self.href.hxe_loss_torch(outputs, batch[1].numpy(), t.perm, t.node_start, t.node_end,
                                        t.tier_base, self.lam)


def _train(rank, world, port, out, clip, steps=2, clip_type="norm", grad_accum=1):
    from hvamd.algorithmic import EMA, GradientClipping
    from hvamd.hierarchy import Taxonomy
    from hvamd.optim import DecoupledSGDW, set_weight_decay
    from hvamd.trainer import Trainer
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    tax = Taxonomy.synthetic(TAX_SIZES)
    model = _OracleSwin(tax)
    opt = DecoupledSGDW(set_weight_decay(model), lr=0.05, momentum=0.9, weight_decay=5e-4)
    ema = EMA(half_life="4ba", update_interval="1ba")
    trainer = Trainer(model, opt, [GradientClipping(clip_type, clip), ema], bucket_mb=0.05,
                      grad_accum=grad_accum)
    if world > 1:
        assert len(trainer.buckets.buckets) > 2  # several all-reduces in flight in the backward
    g = torch.Generator().manual_seed(7)
    x = torch.randn(4, 3, 56, 56, generator=g)
    y = torch.from_numpy(tax.leaf_paths[[1, 5, 9, 11]])
    per = 4 // world
    shard = slice(rank * per, rank * per + per)
    for _ in range(steps):
        trainer.train_step((x[shard], y[shard]))
    out[rank] = ([p.detach().numpy().copy() for p in model.ps],
                 [e.numpy().copy() for e in ema.ema_params])
    if world > 1:
        dist.destroy_process_group()


@pytest.mark.parametrize("clip_type,clip", [("norm", 0.5), ("norm", 1e4), ("value", 2e-3)])
def test_trainer_world2_equals_single_process_full_batch(clip_type, clip):
    """The real Trainer (bucketed hook-driven all-reduce with the 1/world mean handed to
    DecoupledSGDW, GradientClipping handed over as well, EMA every batch) on two gloo ranks
    with half the batch each: parameters and EMA weights after two steps equal one process
    stepping on the whole batch (main.py:44-48 batch split, :104-124 DDP).  Value clipping
    is not handed over: it must see the mean, not the bucket sums (threshold active here)."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_train, args=(2, _free_port(), out, clip, 2, clip_type), nprocs=2, join=True)
    single = {}
    _train(0, 1, 0, single, clip, 2, clip_type)
    for r in range(2):
        for a, b in zip(out[r][0] + out[r][1], single[0][0] + single[0][1]):
            assert torch.allclose(torch.from_numpy(a), torch.from_numpy(b), rtol=1e-4, atol=1e-6), r


@pytest.mark.parametrize("world", [1, 2])
def test_grad_accum_microbatches_equal_one_batch(world):
    """grad_accum = 2 (main.py:121 -> composer's microbatch loop: each microbatch's loss scaled
    by its share, gradients accumulated, DDP's all-reduce only after the last microbatch):
    parameters and EMA weights after two steps equal one process stepping on the whole batch
    with grad_accum = 1.  With two gloo ranks the hook-driven bucket all-reduce must fire once
    per step, after the second microbatch."""
    single = {}
    _train(0, 1, 0, single, 0.5, 2, "norm")
    if world == 1:
        out = {}
        _train(0, 1, 0, out, 0.5, 2, "norm", 2)
    else:
        out = mp.Manager().dict()
        mp.spawn(_train, args=(2, _free_port(), out, 0.5, 2, "norm", 2), nprocs=2, join=True)
    for r in range(world):
        for a, b in zip(out[r][0] + out[r][1], single[0][0] + single[0][1]):
            assert torch.allclose(torch.from_numpy(a), torch.from_numpy(b), rtol=1e-4, atol=1e-6), r


def test_grad_accum_validation():
    """main.py:38-41: "auto" without a GPU is the reference's ValueError; "auto" on the GPU
    resolves to 1; anything but a positive integer raises; a batch that does not split into
    grad_accum equal microbatches raises."""
    from hvamd.trainer import _split_batch, resolve_grad_accum
    with pytest.raises(ValueError, match="requires training with a GPU"):
        resolve_grad_accum("auto", "cpu")
    assert resolve_grad_accum("auto", "cuda") == 1
    assert resolve_grad_accum(4, "cpu") == 4
    for bad in (0, -1, 1.5, "2", True):
        with pytest.raises(ValueError):
            resolve_grad_accum(bad, "cpu")
    x, y = torch.arange(12.0).view(6, 2), torch.arange(6)
    parts = _split_batch((x, y), 3)
    assert [tuple(p[1].tolist()) for p in parts] == [(0, 1), (2, 3), (4, 5)]
    with pytest.raises(ValueError, match="equal microbatches"):
        _split_batch((x, y), 4)


def _train_comm(rank, world, port, out):
    """Trainer.comm_timing on two gloo ranks: every step records the backward's start / end, each
    bucket's all-reduce enqueue and the point after buckets.synchronize(); comm_report turns them
    into the bench line's `comm` fields."""
    from hvamd.algorithmic import GradientClipping
    from hvamd.hierarchy import Taxonomy
    from hvamd.optim import DecoupledSGDW, set_weight_decay
    from hvamd.trainer import Trainer, comm_report
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    tax = Taxonomy.synthetic(TAX_SIZES)
    model = _OracleSwin(tax)
    opt = DecoupledSGDW(set_weight_decay(model), lr=0.05, momentum=0.9, weight_decay=5e-4)
    trainer = Trainer(model, opt, [GradientClipping("norm", 1.0)], bucket_mb=0.05)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(4, 3, 56, 56, generator=g)
    y = torch.from_numpy(tax.leaf_paths[[1, 5, 9, 11]])
    shard = slice(rank * 2, rank * 2 + 2)
    trainer.train_step((x[shard], y[shard]))
    trainer.comm_timing = []
    for _ in range(2):
        trainer.train_step((x[shard], y[shard]))
    rep = comm_report(trainer.comm_timing)
    out[rank] = (rep, len(trainer.buckets.buckets), trainer.buckets.trace)
    dist.destroy_process_group()


def test_comm_timing_world2():
    """The bench's `comm` block on a world-2 gloo run: exposed exchange time >= 0 and shorter than
    a step, one enqueue offset per bucket, all >= 0 (every all-reduce is enqueued before the
    backward ends and at most a backward's length before it)."""
    out = mp.Manager().dict()
    mp.spawn(_train_comm, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        rep, nb, trace = out[r]
        assert trace is None
        assert rep["steps"] == 2 and nb > 2
        assert 0 <= rep["exposed_ms"] <= rep["exposed_ms_max"] < 60_000
        assert rep["backward_ms"] > 0
        offs = rep["bucket_enqueue_before_bwd_end_ms"]
        assert len(offs) == nb and all(o is not None and o >= 0 for o in offs), offs
        assert max(offs) <= rep["backward_ms"] + 1.0
