"""Overlap evidence for the bucketed gradient all-reduce on one GPU: the bench model (SwinV2-T 224
+ HXE) trained by the real Trainer under a ONE-rank RCCL process group with the buckets forced
on (GradientBuckets(force=True)), so every bucket's all_reduce is enqueued from the backward's
post-accumulate-grad hooks exactly as at world > 1.  Run it under a kernel trace:

    rocprofv3 --kernel-trace --output-format csv -d OUT -- python tools/ddp_trace.py
    python tools/ddp_overlap.py OUT        # which RCCL kernels start before the backward ends

--batch sets the images per step (default 64: the same launch sequence, shorter kernels)."""
import argparse
import os
import socket
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    a = ap.parse_args()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    import bench
    from hvamd.ddp import GradientBuckets

    class A:  # bench.build's argument surface
        model, loss, batch = "swinv2_tiny_window7_224", "hxe", a.batch
    cfg, tax, model, trainer = bench.build(A, dev)
    trainer.buckets.remove()
    trainer.buckets = GradientBuckets(model, bucket_mb=a.bucket_mb, force=True)
    print(f"buckets: {len(trainer.buckets.buckets)} "
          f"({', '.join(f'{b[0].numel() * 4 / 2**20:.1f}' for b in trainer.buckets.buckets)} MB)", flush=True)
    batch = bench.synthetic_batch(A, tax, 0, dev)
    # GPU-timeline position of each bucket's all-reduce enqueue (a timing event recorded on the
    # producing stream right before dist.all_reduce: RCCL's stream waits on that point, so the
    # all-reduce can run from there on) against the step's start and the end of the backward
    # (the last bucket's enqueue follows the last gradient)
    sizes = [b[0].numel() * 4 / 2**20 for b in trainer.buckets.buckets]
    for i in range(a.steps):
        torch.cuda.synchronize()
        trainer.buckets.trace = []
        ev0 = torch.cuda.Event(enable_timing=True)
        ev0.record()
        trainer.train_step(batch)
        ev1 = torch.cuda.Event(enable_timing=True)
        ev1.record()
        torch.cuda.synchronize()
        tr, trainer.buckets.trace = trainer.buckets.trace, None
        if i == 0:
            continue  # warm-up
        tend = max(ev0.elapsed_time(e) for _, e in tr)
        print(f"step {i}: step {ev0.elapsed_time(ev1):.2f} ms, backward's last gradient at {tend:.2f} ms")
        for bi, e in tr:
            t = ev0.elapsed_time(e)
            print(f"   bucket {bi} ({sizes[bi]:6.1f} MB) all-reduce enqueued at {t:7.2f} ms = "
                  f"{tend - t:6.2f} ms before the backward ends")
    print("ok", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
