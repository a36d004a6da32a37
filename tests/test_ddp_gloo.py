"""World-size-2 gloo run of the gradient exchange (hvamd.ddp.GradientBuckets) on CPU:
bucketed, hook-driven all-reduce must equal the full-batch gradient of one process."""
import os
import socket

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
