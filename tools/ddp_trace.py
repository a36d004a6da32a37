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
    sizes = [b[0].numel() * 4 / 2**20 for b in trainer.buckets.buckets]
    # GPU-timeline position of each bucket's all-reduce enqueue (a timing mark on the producing
    # stream right before dist.all_reduce: RCCL's stream waits on that point) against the end of
    # the backward, and the exposed exchange after it (Trainer.comm_timing / trainer.comm_report)
    from hvamd.trainer import comm_report
    trainer.train_step(batch)  # warm-up
    trainer.comm_timing = []
    for i in range(a.steps):
        trainer.train_step(batch)
    rep = comm_report(trainer.comm_timing)
    print(rep)
    for bi, off in enumerate(rep["bucket_enqueue_before_bwd_end_ms"]):
        print(f"   bucket {bi} ({sizes[bi]:6.1f} MB) all-reduce enqueued {off} ms before the backward ends")
    print("ok", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
