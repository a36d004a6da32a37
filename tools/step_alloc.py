"""Per-step wall time and caching-allocator growth of the bench step (device mallocs, reserved
bytes), to tell a steady-state step from one that still grows the allocator's pool.

    python tools/step_alloc.py --model swinv2_base_window24_384 --loss hxe --steps 12 [--host-opt k=v]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="swinv2_tiny_window7_224")
    ap.add_argument("--loss", default="hxe")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--host-opt", action="append", default=[])
    args = ap.parse_args()
    import bench
    from hvamd import options
    for o in args.host_opt:
        options.set(**options.parse(o))
    dev = torch.device("cuda:0")
    cfg, tax, model, trainer = bench.build(args, dev)
    batch = bench.synthetic_batch(args, tax, 0, dev, model.module.patch_embed.img_size[0])
    for i in range(args.steps):
        s0 = torch.cuda.memory_stats(dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        trainer.train_step(batch)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        s1 = torch.cuda.memory_stats(dev)
        print(f"step {i:2d} {dt * 1e3:8.1f} ms  device mallocs +{s1.get('num_device_alloc', 0) - s0.get('num_device_alloc', 0):4d}"
              f"  reserved {torch.cuda.memory_reserved(dev) / 2**30:6.1f} GiB  retries {s1.get('num_alloc_retries', 0)}",
              flush=True)


if __name__ == "__main__":
    main()
